#!/bin/bash
# Interleaved A/B (overlapped update, parity-gated by ab_box.sh): the previous commit's
# library (base), the wave_sync build (ws), the working tree (one-wave-per-SIMD forward
# variants at the multi-tile mixers): headline, configs[0]-shape, 64 AGVs.
L=t2omca_amd/lib
timeout -k 10 240 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_mixer_split.py tests/test_gpu_runtime_shapes.py \
  -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r6_check3_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/r6_check3_tests.log)"; [ $rc -ne 0 ] && exit 1
AB_SERIAL= timeout -k 10 500 bash tools/ab_box.sh r6_check3/ab_head $L/libt2omca_base.so $L/libt2omca_ws.so $L/libt2omca.so || exit 1
AB_SERIAL= timeout -k 10 500 bash tools/ab_box.sh r6_check3/ab_a64 $L/libt2omca_base.so $L/libt2omca.so \
  -- --agents 64 --batch 512 --T 60 --steps 3 --warmup 1 || exit 1
AB_SERIAL= timeout -k 10 500 bash tools/ab_box.sh r6_check3/ab_a16 $L/libt2omca_base.so $L/libt2omca.so \
  -- --agents 16 --batch 32 --T 150 || exit 1
exit 0
