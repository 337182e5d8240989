#!/bin/bash
# Run ON THE GPU BOX: the whole -m gpu suite, then the default bench (bf16 + fp32
# companion + CPU baseline legs) -> gpurun_out/<tag>/
set -eu
TAG=${1:-r2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
