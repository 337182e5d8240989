#!/bin/bash
# Run ON THE GPU BOX: interleaved A/B(/C...) bench of several builds of the library,
# serial mode (AB_SERIAL= for the overlapped default), 3 rounds.   tools/ab_box.sh <tag> <lib1.so> <lib2.so> ... [-- bench args]
#   -> gpurun_out/<tag>/<name><round>.json and a median summary on stdout
# Parity gate: each build first runs the configs[2] TD-update parity tests (fp32 +
# bf16 vs the fp64 oracle, tests/test_gpu_configs.py); a build that fails is not
# timed, and every recorded JSON carries "parity": "pass".
set -eu
TAG=$1; shift
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
OK=()
for lib in "${LIBS[@]}"; do
  n=$(basename "$lib" .so)
  if T2O_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q \
       --timeout 120 --timeout-method thread -k config2 > "$OUT/$n.parity.log" 2>&1; then
    OK+=("$lib")
  else
    echo "PARITY FAIL: $n (not timed)"; tail -5 "$OUT/$n.parity.log"
  fi
done
for i in 1 2 3; do
  for lib in "${OK[@]}"; do
    n=$(basename "$lib" .so)
    T2O_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-fp32-companion ${AB_SERIAL---serial} --steps 20 "$@" > "$OUT/$n$i.json"
    python - "$OUT/$n$i.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
d["parity"] = "pass"
json.dump(d, open(sys.argv[1], "w"))
PY
  done
done
python - "$OUT" "${OK[@]}" <<'PY'
import json, os, sys, statistics as st
d = sys.argv[1]
for lib in sys.argv[2:]:
    n = os.path.basename(lib)[:-3]
    rs = [json.load(open(f"{d}/{n}{i}.json")) for i in (1, 2, 3)]
    ks = rs[0]["kernels_ms"].keys()
    print(n, "parity pass, ms/step", [round(r["ms_per_step"], 3) for r in rs],
          {k: round(st.median(r["kernels_ms"][k] for r in rs), 4) for k in ks})
PY
