#!/bin/bash
# The layout-sensitivity hunt on one box, libraries from
# tools/build_debug.sh.  Every step is bounded; test failures (pytest rc 1) are the
# data, anything worse (a crash, a timeout) ends the script.
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
T_KMF="tests/test_gpu_runtime_shapes.py::test_runtime_instance_td_update_fp32 tests/test_gpu_mixer_split.py::test_split_mixer_equals_one_wave_kernels"
T_ODD="tests/test_gpu_mixer_split.py tests/test_gpu_reproducibility.py tests/test_gpu_runtime_shapes.py::test_runtime_instance_td_update_fp32"
T_PF="tests/test_gpu_reproducibility.py"
case "${1:-all}" in
  all)
    step e1_product_poison "" 1 tests/
    step e2_dbg_poison dbg 1 tests/
    for v in kmf odd pf; do
      eval T=\$T_$(echo $v | tr a-z A-Z)
      step e3_$v $v 0 $T
      step e4_dbg_$v dbg_$v 1 $T
    done
    for v in pf dbg_pf odd; do
      T2O_LIB=$L/$v.so timeout -k 10 300 python -u tools/diag_repro.py --repeats 10 8,64,12,bf16 16,4,6,bf16 \
        > $OUT/e5_repro_$v.log 2>&1
      rc=$?; echo "e5_repro_$v rc=$rc"; tail -3 $OUT/e5_repro_$v.log
      [ $rc -gt 1 ] && exit $rc
    done
    ;;
  two)  # after the first pass: which poison reaches the flat-mask failure; the odd-pair fixes;
        # run-to-run stress of the product and the pair-full contraction
    step x1_kmf_pypoison kmf 1 $T_KMF
    for v in odd2 odd3; do
      step x2_$v $v 0 $T_ODD
      T2O_LIB=$L/$v.so timeout -k 10 300 python -u tools/diag_repro.py --repeats 10 16,4,6,bf16 64,2,3,bf16 \
        > $OUT/x2_repro_$v.log 2>&1
      rc=$?; echo "x2_repro_$v rc=$rc"; tail -2 $OUT/x2_repro_$v.log
      [ $rc -gt 1 ] && exit $rc
    done
    for v in libt2omca pf; do
      T2O_LIB=$L/$v.so timeout -k 10 400 python -u tools/diag_repro.py --repeats 30 8,64,12,bf16 16,4,6,bf16 \
        8,1024,60,bf16 > $OUT/x3_stress_$v.log 2>&1
      rc=$?; echo "x3_stress_$v rc=$rc"; tail -3 $OUT/x3_stress_$v.log
      [ $rc -gt 1 ] && exit $rc
    done
    timeout -k 10 400 python -u -m pytest -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider \
      tests/test_gpu_fullgrid.py > $OUT/x4_fullgrid.log 2>&1
    rc=$?; echo "x4_fullgrid rc=$rc $(tail -1 $OUT/x4_fullgrid.log)"
    ;;
esac
exit 0
