#!/bin/bash
# Run ON THE GPU BOX: A/B bench of the baseline library (t2omca_amd/lib/libt2omca_base.so)
# against the current one, interleaved 3 times, serial mode, bf16.  -> gpurun_out/<tag>/ab.txt
set -eu
TAG=${1:-ab}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for i in 1 2 3; do
  for v in base cur; do
    lib=t2omca_amd/lib/libt2omca.so; [ $v = base ] && lib=t2omca_amd/lib/libt2omca_base.so
    T2O_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --serial --steps 20 "$@" > "$OUT/$v$i.json"
  done
done
python - "$OUT" <<'PY'
import json, sys, statistics as st
d = sys.argv[1]
for v in ("base", "cur"):
    rs = [json.load(open(f"{d}/{v}{i}.json")) for i in (1, 2, 3)]
    ks = rs[0]["kernels_ms"].keys()
    print(v, "ms/step", [round(r["ms_per_step"], 3) for r in rs],
          {k: round(st.median(r["kernels_ms"][k] for r in rs), 4) for k in ks})
PY
