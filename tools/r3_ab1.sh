#!/bin/bash
# Run ON THE GPU BOX: A=40 seed-3 diagnostic (ReLU margin), then the interleaved
# overlapped A/B of: session start, runtime instances, + ordered flush & padded rows, and
# the same without the ordered flush.
set -u
mkdir -p gpurun_out/r3_ab1
DIAG_SEED=3 timeout -k 10 120 python tools/diag_rt.py 40 1 4 > gpurun_out/r3_ab1/diag3.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r3_ab1/diag3.log | sed -n 1,4p
AB_SERIAL= bash tools/ab_box.sh r3_ab1 t2omca_amd/lib/libt2omca_s0.so t2omca_amd/lib/libt2omca_rt.so \
  t2omca_amd/lib/libt2omca.so t2omca_amd/lib/libt2omca_nondet.so
