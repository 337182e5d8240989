#!/bin/bash
# Run ON THE GPU BOX: interleaved rollout-bench A/B of env-kernel builds (configs[4]
# shape, 8192 envs x 16 AGVs x T=150), 3 rounds:  tools/env_ab_box.sh <tag> <lib.so> ...
set -eu
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for i in 1 2 3; do
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    T2O_LIB=$PWD/$lib timeout -k 10 200 python bench.py --mode rollout --steps 3 --warmup 1 --no-cpu-baseline \
      --kernel-timer-every 1 > "$OUT/$n$i.json"
  done
done
python - "$OUT" "$@" <<'PY'
import json, os, sys, statistics as st
d = sys.argv[1]
for lib in sys.argv[2:]:
    n = os.path.basename(lib)[:-3]
    rs = [json.load(open(f"{d}/{n}{i}.json")) for i in (1, 2, 3)]
    print(n, "per env step ms", [round(r["per_env_step_ms"], 4) for r in rs],
          {k: round(st.median(r["kernels_ms"][k] for r in rs), 4) for k in rs[0]["kernels_ms"]})
PY
