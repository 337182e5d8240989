#!/bin/bash
# Run ON THE GPU BOX: GPU suite, headline bench (no CPU legs), 64-AGV config, softplus head.
set -u
OUT=gpurun_out/${1:-r3_chk}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; grep -E "^FAILED|passed|failed" "$OUT/pytest.log" | tail -12; [ $rc -ge 124 ] && exit 1
B="timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-companion"
$B > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
$B --agents 64 --batch 512 --T 60 --steps 3 --warmup 1 > "$OUT/c4_train.json" 2> "$OUT/c4.err" || { tail -5 "$OUT/c4.err"; exit 1; }
$B --qmix-pos-func softplus > "$OUT/softplus.json" 2> "$OUT/softplus.err" || { tail -5 "$OUT/softplus.err"; exit 1; }
for f in "$OUT"/*.json; do
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d['value']/1e6,2),'M/s',round(d['ms_per_step'],3),'ms',d['dtype'],d['config'].get('kernels'),d['kernels_ms'])" "$f"
done
