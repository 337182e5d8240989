#!/bin/bash
# Round-6 check 2: does the flat fp32 key mask pass once every intra-wave LDS hand-off
# is a compiler ordering point (wave_sync)?  Then the GPU suite on the product and an
# interleaved A/B of the product against the previous commit's build (headline).
OUT=gpurun_out/r6_check2; mkdir -p $OUT
L=$PWD/t2omca_amd/lib
T_KMF="tests/test_gpu_runtime_shapes.py::test_runtime_instance_td_update_fp32 tests/test_gpu_mixer_split.py::test_split_mixer_equals_one_wave_kernels tests/test_gpu_reproducibility.py"
T2O_LIB=$L/kmfw.so timeout -k 10 400 python -u -m pytest -m gpu -q -s --timeout 120 --timeout-method thread \
  -p no:cacheprovider $T_KMF > $OUT/kmfw.log 2>&1
rc=$?; echo "kmfw rc=$rc $(tail -1 $OUT/kmfw.log)"; grep "^FAILED" $OUT/kmfw.log | head; [ $rc -gt 1 ] && exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest.log 2>&1
rc=$?; echo "suite rc=$rc $(tail -1 $OUT/pytest.log)"; grep "^FAILED" $OUT/pytest.log | head; [ $rc -gt 1 ] && exit 1
AB_SERIAL= timeout -k 10 600 bash tools/ab_box.sh r6_check2/ab_head $L/libt2omca_base.so $L/libt2omca.so || exit 1
exit 0
