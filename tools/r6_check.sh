#!/bin/bash
# Round-6 mid-round check on one box: the GPU suite on the product library (ABI 6),
# then the odd key-tile pairing forms against the unpaired default (interleaved A/B,
# overlapped update): configs[0]-shape (16 AGVs, 32 x 150) and 64 AGVs (512 x 60).
OUT=gpurun_out/r6_check; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; grep "^FAILED" $OUT/pytest.log | head; [ $rc -gt 1 ] && exit 1
L=t2omca_amd/lib
AB_SERIAL= timeout -k 10 600 bash tools/ab_box.sh r6_check/ab_a16 $L/libt2omca.so $L/odd2.so $L/odd3.so \
  -- --agents 16 --batch 32 --T 150 || exit 1
AB_SERIAL= timeout -k 10 600 bash tools/ab_box.sh r6_check/ab_a64 $L/libt2omca.so $L/odd2.so $L/odd3.so \
  -- --agents 64 --batch 512 --T 60 --steps 3 --warmup 1 || exit 1
exit 0
