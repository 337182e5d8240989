#!/bin/bash
# Run ON THE GPU BOX: ablation timings (no parity gate: an ablation computes wrong
# gradients on purpose), serial mode, interleaved, 2 rounds.
#   tools/r3_abl.sh <tag> <lib1.so> <lib2.so> ...
set -eu
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for i in 1 2; do
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    T2O_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-fp32-companion --serial --steps 20 > "$OUT/$n$i.json"
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d['ms_per_step'],4),d['kernels_ms'])" "$OUT/$n$i.json"
  done
done
