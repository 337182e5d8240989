#!/bin/bash
# Run ON THE GPU BOX: the runtime-entity instances' parity tests first, then the
# whole GPU suite, the default bench line (no CPU legs) and train bench lines at
# AGV counts without an exact instance.
#   tools/r3_rt.sh <tag> [agents...]  -> gpurun_out/<tag>/
set -eu
TAG=${1:-r3_rt}
shift || true
AGENTS=${*:-12 32}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_runtime_shapes.py -m gpu -x -v -s --timeout 120 \
  --timeout-method thread > "$OUT/pytest_rt.log" 2>&1 || { tail -40 "$OUT/pytest_rt.log"; exit 1; }
grep -E "PASS|FAIL|A[0-9]+ (fp32|bf16)" "$OUT/pytest_rt.log" | cut -c1-200 | tail -40
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { tail -20 "$OUT/bench.err"; exit 1; }
cut -c1-700 "$OUT/bench.json"
for A in $AGENTS; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-companion --agents "$A" > "$OUT/bench_a$A.json" \
    2> "$OUT/bench_a$A.err" || { tail -20 "$OUT/bench_a$A.err"; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms', d['config']['kernels'], d['dtype'], d['kernels_ms'])" "$OUT/bench_a$A.json" "A=$A"
done
