#!/bin/bash
# Run ON THE GPU BOX: interleaved A/B of environment-variable variants of the
# default bench (overlapped), 3 rounds.   tools/r3_envab.sh <tag> "VAR=a" "VAR=b" ...
set -eu
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for i in 1 2 3; do
  k=0
  for v in "$@"; do
    k=$((k+1))
    env $v timeout -k 10 200 python bench.py --no-cpu-baseline --no-fp32-companion --steps 20 > "$OUT/v$k.$i.json"
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],round(d['ms_per_step'],4))" "$OUT/v$k.$i.json" "$v"
  done
done
