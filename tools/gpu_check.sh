#!/bin/bash
# Run ON THE GPU BOX: GPU parity tests, then the bench in bf16 and fp32 (no CPU leg).
#   tools/gpu_check.sh [tag]    -> gpurun_out/<tag>/{pytest.log,bench_bf16.json,bench_fp32.json}
set -eu
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 200 python bench.py --no-cpu-baseline > "$OUT/bench_bf16.json" 2> "$OUT/bench_bf16.err"
timeout -k 10 200 python bench.py --no-cpu-baseline --dtype fp32 > "$OUT/bench_fp32.json" 2> "$OUT/bench_fp32.err"
timeout -k 10 200 python bench.py --no-cpu-baseline --serial > "$OUT/bench_bf16_serial.json" 2> "$OUT/bench_bf16_serial.err"
python - "$OUT" <<'PY'
import json, sys
for d in ("bf16", "fp32", "bf16_serial"):
    r = json.load(open(f"{sys.argv[1]}/bench_{d}.json"))
    print(d, f"{r['value']/1e6:.2f}M/s", f"{r['ms_per_step']:.3f} ms", r["kernels_ms"])
PY
