#!/bin/bash
# Run ON THE GPU BOX: per-parameter gradient errors of the runtime-entity instances.
set -u
OUT=gpurun_out/r3_diag4
mkdir -p $OUT
for s in 4 5 6; do
  for cfg in "40 1 4" "24 1 4" "56 1 3" "32 1 4"; do
    DIAG_SEED=$s timeout -k 10 120 python tools/diag_rt.py $cfg >> $OUT/diag.log 2>&1 || { tail -20 $OUT/diag.log; exit 1; }
  done
done
grep -v amdgpu.ids $OUT/diag.log | grep -A1 "^A="
