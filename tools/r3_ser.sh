#!/bin/bash
# Run ON THE GPU BOX: overlapped (side-stream mixer contraction) vs serial update, interleaved, 3 rounds.
set -u
OUT=gpurun_out/r3_ser
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-fp32-companion --steps 20 > $OUT/ovl$i.json || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-fp32-companion --steps 20 --serial > $OUT/ser$i.json || exit 1
done
for m in ovl ser; do
  python - $OUT $m <<'PY'
import json, sys, statistics as st
d, m = sys.argv[1:3]
rs = [json.load(open(f"{d}/{m}{i}.json")) for i in (1, 2, 3)]
print(m, [round(r["ms_per_step"], 3) for r in rs], {k: round(st.median(r["kernels_ms"][k] for r in rs), 4) for k in rs[0]["kernels_ms"]})
PY
done
