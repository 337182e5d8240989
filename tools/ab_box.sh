#!/bin/bash
# Run ON THE GPU BOX: interleaved A/B(/C...) bench of several builds of the library,
# serial mode (AB_SERIAL= for the overlapped default), 3 rounds.   tools/ab_box.sh <tag> <lib1.so> <lib2.so> ... [-- bench args]
#   -> gpurun_out/<tag>/<name><round>.json and a median summary on stdout
set -eu
TAG=$1; shift
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for i in 1 2 3; do
  for lib in "${LIBS[@]}"; do
    n=$(basename "$lib" .so)
    T2O_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-fp32-companion ${AB_SERIAL---serial} --steps 20 "$@" > "$OUT/$n$i.json"
  done
done
python - "$OUT" "${LIBS[@]}" <<'PY'
import json, os, sys, statistics as st
d = sys.argv[1]
for lib in sys.argv[2:]:
    n = os.path.basename(lib)[:-3]
    rs = [json.load(open(f"{d}/{n}{i}.json")) for i in (1, 2, 3)]
    ks = rs[0]["kernels_ms"].keys()
    print(n, "ms/step", [round(r["ms_per_step"], 3) for r in rs],
          {k: round(st.median(r["kernels_ms"][k] for r in rs), 4) for k in ks})
PY
