# full GPU suite twice per library (the current one and the one before the paired contraction):
# is the one reproducibility failure of r5_final2 tied to the pairing?
set -u
OUT=gpurun_out/r5_flaky; mkdir -p $OUT
for i in 1 2; do
  for v in cur prepair; do
    T2O_LIB=$PWD/t2omca_amd/lib/ab_$v.so timeout -k 10 400 python -u -m pytest tests -m gpu -q -s --timeout 120 --timeout-method thread > $OUT/${v}_$i.log 2>&1
    rc=$?; echo "$v run $i rc=$rc: $(tail -1 $OUT/${v}_$i.log)"; grep -A2 "differing indices\|^FAILED" $OUT/${v}_$i.log | head -8
    [ $rc -ge 124 ] && exit 1
  done
done
exit 0
