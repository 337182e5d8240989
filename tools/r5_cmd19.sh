# reproducibility failure rate: the library before the paired contraction vs the current one
set -u
OUT=gpurun_out/r5_rep; mkdir -p $OUT
for v in prepair cur; do
  for i in 1 2 3 4; do
    T2O_LIB=$PWD/t2omca_amd/lib/ab_$v.so timeout -k 10 120 python -u -m pytest -q -s --timeout 100 --timeout-method thread -m gpu \
      "tests/test_gpu_reproducibility.py::test_td_update_bit_reproducible_across_runs[8-64-12-bf16]" \
      "tests/test_gpu_reproducibility.py::test_paired_contraction_equals_separate_launches[8-64-12-bf16]" > $OUT/${v}_$i.log 2>&1
    rc=$?; echo "$v run $i rc=$rc $(grep -o 'grad: [0-9]* differing' $OUT/${v}_$i.log | tr '\n' ' ')"
    [ $rc -ge 124 ] && exit 1
  done
done
exit 0
