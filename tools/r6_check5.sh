#!/bin/bash
# Mixer weight placement by resident waves per CU (mix_pick) against the previous build
# (km): fp32 16 AGVs (1024 x 150; configs[0]-shape 32 x 150), 64 AGVs bf16 / fp32,
# headline; GPU mixer tests on the new build first.
OUT=gpurun_out/r6_check5; mkdir -p $OUT
L=t2omca_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_mixer.py tests/test_gpu_mixer_split.py tests/test_gpu_configs.py \
  tests/test_gpu_runtime_shapes.py tests/test_gpu_reproducibility.py -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"; [ $rc -ne 0 ] && exit 1
AB_SERIAL= timeout -k 10 500 bash tools/ab_box.sh r6_check5/ab_a16f $L/libt2omca_km.so $L/libt2omca.so \
  -- --agents 16 --batch 1024 --T 150 --steps 3 --warmup 1 --dtype fp32 || exit 1
AB_SERIAL= timeout -k 10 500 bash tools/ab_box.sh r6_check5/ab_c0f $L/libt2omca_km.so $L/libt2omca.so \
  -- --agents 16 --batch 32 --T 150 --dtype fp32 || exit 1
AB_SERIAL= timeout -k 10 500 bash tools/ab_box.sh r6_check5/ab_a64 $L/libt2omca_km.so $L/libt2omca.so \
  -- --agents 64 --batch 512 --T 60 --steps 3 --warmup 1 || exit 1
AB_SERIAL= timeout -k 10 500 bash tools/ab_box.sh r6_check5/ab_a64f $L/libt2omca_km.so $L/libt2omca.so \
  -- --agents 64 --batch 512 --T 60 --steps 2 --warmup 1 --dtype fp32 || exit 1
AB_SERIAL= timeout -k 10 300 bash tools/ab_box.sh r6_check5/ab_head $L/libt2omca_km.so $L/libt2omca.so || exit 1
exit 0
