#!/bin/bash
# Run ON THE GPU BOX: GPU suite on the working build, then interleaved overlapped
# A/B (bf16 headline) and a serial fp32 A/B of HEAD vs the working build.
set -u
mkdir -p gpurun_out/r3_ab5
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3_ab5/pytest.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed" gpurun_out/r3_ab5/pytest.log | tail -12; [ $rc -ge 124 ] && exit 1
AB_SERIAL= bash tools/ab_box.sh r3_ab5 t2omca_amd/lib/libt2omca_h2.so t2omca_amd/lib/libt2omca.so
bash tools/ab_box.sh r3_ab5f t2omca_amd/lib/libt2omca_h2.so t2omca_amd/lib/libt2omca.so -- --dtype fp32
