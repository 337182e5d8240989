# bisect the multi-tile bf16 mixer backward failure over library variants
set -u
OUT=gpurun_out/r5_bis; mkdir -p $OUT
for v in base v1 v2 new; do
  T2O_LIB=$PWD/t2omca_amd/lib/ab_$v.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_mixer_split.py tests/test_gpu_reproducibility.py "tests/test_gpu_runtime_shapes.py::test_runtime_instance_td_update_fp32" > $OUT/$v.log 2>&1
  rc=$?; echo "== $v rc=$rc: $(tail -1 $OUT/$v.log)"; grep FAILED $OUT/$v.log | cut -c1-120
  [ $rc -ge 124 ] && exit 1
done
exit 0
