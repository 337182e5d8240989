#!/bin/bash
# Run ON THE GPU BOX: the -m gpu suite on the working-tree library, the default
# bench line, then an interleaved A/B of two library builds.
#   tools/gpu_ab.sh <tag> <libA.so> <libB.so>   -> gpurun_out/<tag>/
set -eu
TAG=$1; A=$2; B=$3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 240 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(round(d['value']/1e6,2),round(d['ms_per_step'],3),d['kernels_ms'])" "$OUT/bench.json"
bash tools/ab_box.sh "${TAG}_ab" "$A" "$B"
