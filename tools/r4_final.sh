#!/bin/bash
# Run ON THE GPU BOX: the round's evidence on one build — GPU suite, smoke, the
# driver-equivalent default bench line (CPU legs included), kernel-trace stats +
# HBM traffic of the default workload, the rollout line, the other BASELINE
# configs, runtime-entity shapes (and the generic kernels on one of them for
# comparison) and the headline shape with a softplus mixer head.
#   tools/r4_final.sh <tag>  -> gpurun_out/<tag>/
set -u
TAG=${1:-r4_final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() { echo "== $1"; }
step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -1 "$OUT/pytest.log"; [ $rc -ge 124 ] && exit 1
step smoke
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
step bench
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
cut -c1-300 "$OUT/bench.json"
step profile
bash tools/profile_box.sh "$TAG/prof" > "$OUT/prof.log" 2>&1 || { tail -5 "$OUT/prof.log"; exit 1; }
python3 tools/timeline_trace.py $(find "$OUT/prof/trace" -name "*kernel_trace.csv" | head -1) > "$OUT/prof/timeline.txt"
tail -1 "$OUT/prof/timeline.txt"
step rollout
timeout -k 10 300 python bench.py --mode rollout > "$OUT/rollout.json" 2> "$OUT/rollout.err" || { tail -5 "$OUT/rollout.err"; exit 1; }
timeout -k 10 300 python bench.py --mode rollout --rollout-precision bf16 > "$OUT/rollout_bf16.json" 2> "$OUT/rollout_bf16.err" || { tail -5 "$OUT/rollout_bf16.err"; exit 1; }
for f in "$OUT"/rollout.json "$OUT"/rollout_bf16.json; do
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d['value']/1e6,1),'M/s',d['kernels_ms'])" "$f"
done
step dropin
timeout -k 10 300 python bench.py --mode dropin > "$OUT/dropin.json" 2> "$OUT/dropin.err" || { tail -5 "$OUT/dropin.err"; exit 1; }
step loop
timeout -k 10 300 python bench.py --mode loop --steps 3 --warmup 1 > "$OUT/loop.json" 2> "$OUT/loop.err" || { tail -5 "$OUT/loop.err"; exit 1; }
step configs
bash tools/configs_box.sh "$TAG/configs" > "$OUT/configs.log" 2>&1 || { tail -5 "$OUT/configs.log"; exit 1; }
cat "$OUT/configs.log"
step shapes
for A in 12 32; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-companion --agents $A > "$OUT/a$A.json" 2> "$OUT/a$A.err" \
    || { tail -5 "$OUT/a$A.err"; exit 1; }
done
T2O_GENERIC=1 timeout -k 10 400 python bench.py --no-cpu-baseline --no-fp32-companion --agents 32 --steps 3 --warmup 1 \
  > "$OUT/a32_generic.json" 2> "$OUT/a32_generic.err" || { tail -5 "$OUT/a32_generic.err"; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-companion --qmix-pos-func softplus \
  > "$OUT/softplus.json" 2> "$OUT/softplus.err" || { tail -5 "$OUT/softplus.err"; exit 1; }
for f in "$OUT"/a*.json "$OUT"/softplus.json; do
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d['value']/1e6,2),'M/s',round(d['ms_per_step'],3),'ms',d['dtype'],d['config'].get('kernels'),d['kernels_ms'])" "$f"
done
