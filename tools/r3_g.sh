#!/bin/bash
# Run ON THE GPU BOX: GPU suite, then the rollout line and the drop-in per-call line.
#   tools/r3_g.sh <tag>  -> gpurun_out/<tag>/
set -u
TAG=${1:-r3_g}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
echo "== pytest"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit 1
echo "== rollout"
timeout -k 10 300 python bench.py --mode rollout --no-cpu-baseline > "$OUT/rollout.json" 2> "$OUT/rollout.err" || { tail -5 "$OUT/rollout.err"; exit 1; }
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['ms_per_step'],d['per_env_step_ms'],d['kernels_ms'])" "$OUT/rollout.json"
echo "== rollout wire"
timeout -k 10 300 python bench.py --mode rollout --no-cpu-baseline --compact-obs > "$OUT/rollout_wire.json" 2> "$OUT/rollout_wire.err" || { tail -5 "$OUT/rollout_wire.err"; exit 1; }
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['ms_per_step'],d['per_env_step_ms'],d['kernels_ms'])" "$OUT/rollout_wire.json"
echo "== dropin"
timeout -k 10 300 python bench.py --mode dropin > "$OUT/dropin.json" 2> "$OUT/dropin.err" || { tail -5 "$OUT/dropin.err"; exit 1; }
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(json.dumps(d['per_call_ms']), d['pack_rebuilds'])" "$OUT/dropin.json"
