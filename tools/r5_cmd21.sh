# agent-record-only pairing: full GPU suite twice, then A/B against the pre-pair library
set -u
OUT=gpurun_out/r5_pa; mkdir -p $OUT
for i in 1 2; do
  T2O_LIB=$PWD/t2omca_amd/lib/ab_pa.so timeout -k 10 400 python -u -m pytest tests -m gpu -q -s --timeout 120 --timeout-method thread > $OUT/suite_$i.log 2>&1
  rc=$?; echo "suite $i rc=$rc: $(tail -1 $OUT/suite_$i.log)"; grep -A2 "differing indices\|^FAILED" $OUT/suite_$i.log | head -8
  [ $rc -ne 0 ] && exit 1
done
AB_SERIAL= bash tools/ab_box.sh r5_pa/head t2omca_amd/lib/ab_prepair.so t2omca_amd/lib/ab_pa.so || exit 1
