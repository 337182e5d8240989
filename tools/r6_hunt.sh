#!/bin/bash
# The poisoned-build pass of the layout-sensitivity hunt on one
# box, with tools/build_debug.sh's dbg.so.  Every step is bounded; test failures
# (pytest rc 1) are the data, anything worse (a crash, a timeout) ends the script.
# (Round 6 ran the per-form passes here too, against builds with the switches that
# DESIGN.md §2d records as deleted; gpurun_out/r6_hunt logs and profiles/r6_hunt keep them.)
OUT=gpurun_out/r6_hunt; mkdir -p $OUT
L=$PWD/t2omca_amd/lib
PYT="python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider"
step() {  # step <name> <lib or ""> <poison 0/1> <pytest args...>
  local name=$1 lib=$2 poison=$3; shift 3
  local env=(T2O_POISON=$poison)
  [ -n "$lib" ] && env+=(T2O_LIB=$L/$lib.so)
  env "${env[@]}" timeout -k 10 ${STEP_TIMEOUT:-420} $PYT "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -1 $OUT/$name.log)"; grep "^FAILED" $OUT/$name.log | head -20
  [ $rc -gt 1 ] && exit $rc
  return 0
}
step e1_product_poison "" 1 tests/
step e2_dbg_poison dbg 1 tests/
for v in libt2omca dbg; do
  T2O_LIB=$L/$v.so timeout -k 10 400 python -u tools/diag_repro.py --repeats 30 8,64,12,bf16 16,4,6,bf16 \
    8,1024,60,bf16 > $OUT/x3_stress_$v.log 2>&1
  rc=$?; echo "x3_stress_$v rc=$rc"; tail -3 $OUT/x3_stress_$v.log
  [ $rc -gt 1 ] && exit $rc
done
exit 0
