#!/bin/bash
# Run ON THE GPU BOX: bench.py --gpus 2 started as a plain process (the driver's SCALE
# invocation) with the two ranks sharing the one GPU over gloo.
set -eu
OUT=gpurun_out/${1:-dp2}
mkdir -p "$OUT"
T2O_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --no-fp32-companion \
  > "$OUT/bench_dp2_gloo.json" 2> "$OUT/bench_dp2_gloo.err" || { tail -30 "$OUT/bench_dp2_gloo.err"; exit 1; }
cat "$OUT/bench_dp2_gloo.json"
