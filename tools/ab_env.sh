#!/bin/bash
# Run ON THE GPU BOX: interleaved A/B of environment settings on one library build,
# serial mode, 3 rounds.   tools/ab_env.sh <tag> "<ENV=a ...>" "<ENV=b ...>" ... [-- bench args]
#   -> gpurun_out/<tag>/v<k>_<round>.json and a median summary on stdout
set -eu
TAG=$1; shift
VARS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for i in 1 2 3; do
  for k in "${!VARS[@]}"; do
    env ${VARS[$k]} timeout -k 10 200 python bench.py --no-cpu-baseline --serial --steps 20 "$@" > "$OUT/v${k}_$i.json"
  done
done
python - "$OUT" "${VARS[@]}" <<'PY'
import json, sys, statistics as st
d = sys.argv[1]
for k, v in enumerate(sys.argv[2:]):
    rs = [json.load(open(f"{d}/v{k}_{i}.json")) for i in (1, 2, 3)]
    ks = rs[0]["kernels_ms"].keys()
    print(repr(v), "ms/step", [round(r["ms_per_step"], 3) for r in rs],
          {k2: round(st.median(r["kernels_ms"][k2] for r in rs), 4) for k2 in ks})
PY
