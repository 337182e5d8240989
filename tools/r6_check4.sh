#!/bin/bash
# GPU suite on the product (LDS-read fp32 key fragments at KT >= 5, opaque weight views
# per query tile), the flat fp32 key mask on the same code (kmfx), and interleaved A/B
# against the previous build (lb): 64 AGVs bf16 and fp32, 16 AGVs fp32, headline.
OUT=gpurun_out/r6_check4; mkdir -p $OUT
L=t2omca_amd/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest.log 2>&1
rc=$?; echo "suite rc=$rc $(tail -1 $OUT/pytest.log)"; grep "^FAILED" $OUT/pytest.log | head; [ $rc -gt 1 ] && exit 1
T_KMF="tests/test_gpu_runtime_shapes.py::test_runtime_instance_td_update_fp32 tests/test_gpu_mixer_split.py::test_split_mixer_equals_one_wave_kernels tests/test_gpu_reproducibility.py"
T2O_LIB=$PWD/$L/kmfx.so timeout -k 10 400 python -u -m pytest -m gpu -q -s --timeout 120 --timeout-method thread \
  -p no:cacheprovider $T_KMF > $OUT/kmfx.log 2>&1
rc=$?; echo "kmfx rc=$rc $(tail -1 $OUT/kmfx.log)"; grep "^FAILED" $OUT/kmfx.log | head; [ $rc -gt 1 ] && exit 1
AB_SERIAL= timeout -k 10 500 bash tools/ab_box.sh r6_check4/ab_a64 $L/libt2omca_lb.so $L/libt2omca.so \
  -- --agents 64 --batch 512 --T 60 --steps 3 --warmup 1 || exit 1
AB_SERIAL= timeout -k 10 500 bash tools/ab_box.sh r6_check4/ab_a64f $L/libt2omca_lb.so $L/libt2omca.so \
  -- --agents 64 --batch 512 --T 60 --steps 2 --warmup 1 --dtype fp32 || exit 1
AB_SERIAL= timeout -k 10 500 bash tools/ab_box.sh r6_check4/ab_a16f $L/libt2omca_lb.so $L/libt2omca.so \
  -- --agents 16 --batch 1024 --T 150 --steps 3 --warmup 1 --dtype fp32 || exit 1
AB_SERIAL= timeout -k 10 500 bash tools/ab_box.sh r6_check4/ab_head $L/libt2omca_lb.so $L/libt2omca.so || exit 1
exit 0
