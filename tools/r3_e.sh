#!/bin/bash
# Run ON THE GPU BOX: GPU suite, default bench (no CPU legs), then the other configs.
set -eu
TAG=${1:-r3_e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 \
  || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(round(d['value']/1e6,2), round(d['ms_per_step'],4), d['kernels_ms'])"
bash tools/configs_box.sh $TAG/configs
