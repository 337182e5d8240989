#!/bin/bash
# Run ON THE GPU BOX: the GPU suite on the working build, then an interleaved
# overlapped A/B: runtime-instances build / previous HEAD / working build.
set -u
mkdir -p gpurun_out/r3_ab3
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s --timeout 120 --timeout-method thread \
  > gpurun_out/r3_ab3/pytest.log 2>&1
rc=$?
if [ $rc -ge 124 ]; then tail -30 gpurun_out/r3_ab3/pytest.log; exit 1; fi
grep -E "^FAILED|passed|failed" gpurun_out/r3_ab3/pytest.log | tail -20
AB_SERIAL= bash tools/ab_box.sh r3_ab3 t2omca_amd/lib/libt2omca_rt.so t2omca_amd/lib/libt2omca_h1.so \
  t2omca_amd/lib/libt2omca.so
