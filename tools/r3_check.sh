#!/bin/bash
# Run ON THE GPU BOX: the GPU suite, smoke(), then the driver's default bench line.
#   tools/r3_check.sh <tag> [pytest -k expr]  -> gpurun_out/<tag>/{pytest.log,smoke.log,bench.json}
set -eu
TAG=${1:-check}
K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ -n "$K" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" \
    > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
else
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
fi
tail -3 "$OUT/pytest.log"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  || { tail -20 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
