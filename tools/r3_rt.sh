#!/bin/bash
# Run ON THE GPU BOX: the whole GPU suite (no -x: every failure listed), the
# A=40 diagnostics, the default bench line (no CPU legs) and train bench lines at
# AGV counts without an exact instance.
#   tools/r3_rt.sh <tag> [agents...]  -> gpurun_out/<tag>/
set -u
TAG=${1:-r3_rt}
shift || true
AGENTS=${*:-12 32}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s --timeout 120 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1
rc=$?
if [ $rc -ge 124 ]; then tail -30 "$OUT/pytest.log"; exit 1; fi
grep -E "^FAILED|passed|failed" "$OUT/pytest.log" | tail -30
for s in 4 5; do
  DIAG_SEED=$s timeout -k 10 120 python tools/diag_rt.py 40 1 4 > "$OUT/diag_$s.log" 2>&1 || exit 1
  grep -v amdgpu.ids "$OUT/diag_$s.log" | sed -n 1,4p
done
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { tail -20 "$OUT/bench.err"; exit 1; }
cut -c1-600 "$OUT/bench.json"
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['kernels_ms'])" "$OUT/bench.json"
for A in $AGENTS; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-companion --agents "$A" > "$OUT/bench_a$A.json" \
    2> "$OUT/bench_a$A.err" || { tail -20 "$OUT/bench_a$A.err"; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms', d['config']['kernels'], d['dtype'], d['kernels_ms'])" "$OUT/bench_a$A.json" "A=$A"
done
