#!/bin/bash
# Run ON THE GPU BOX: mixer-related GPU tests, then kernel-trace stats of the
# multi-tile mixer configs (A=16 T=150, A=64 T=60) -> gpurun_out/<tag>/
set -eu
OUT=gpurun_out/$1
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_learner.py tests/test_gpu_mixer.py -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/a16" -o run -- python bench.py --no-cpu-baseline --no-fp32-companion --agents 16 --batch 1024 --T 150 --steps 5 > "$OUT/a16.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/a64" -o run -- python bench.py --no-cpu-baseline --no-fp32-companion --agents 64 --batch 512 --T 60 --steps 3 --warmup 1 > "$OUT/a64.json"
cat "$OUT"/a16.json "$OUT"/a64.json
