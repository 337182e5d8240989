# Localise the fp32 capacity-64 failure of the flat key mask (T2O_KM_FP32_FLAT):
# each library differs from the default in one source's mask form; run the two tests that failed.
OUT=gpurun_out/r5_kmf; mkdir -p $OUT
for v in ${KMF_VARIANTS:-kf_m3 kf_s3 kf_m1 kf_m2}; do
  T2O_LIB=$PWD/t2omca_amd/lib/$v.so timeout -k 10 240 python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread \
    "tests/test_gpu_runtime_shapes.py::test_runtime_instance_td_update_fp32" "tests/test_gpu_mixer_split.py::test_split_mixer_equals_one_wave_kernels" \
    > $OUT/$v.log 2>&1
  rc=$?; echo "$v rc=$rc $(tail -1 $OUT/$v.log)"; grep "^FAILED" $OUT/$v.log
  [ $rc -gt 1 ] && exit 1
done
exit 0
