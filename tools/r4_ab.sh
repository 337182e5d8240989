#!/bin/bash
# Run ON THE GPU BOX: interleaved A/B of library builds (tools/ab_box.sh, serial),
# then the softplus-head headline on the newest build and the parity suites the
# round's kernel changes touch.   tools/r4_ab.sh <tag> <lib.so>...
set -u
TAG=$1; shift
bash tools/ab_box.sh "$TAG" "$@" || exit 1
OUT=gpurun_out/$TAG
timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-companion --qmix-pos-func softplus > "$OUT/softplus.json" 2> "$OUT/softplus.err" \
  || { tail -5 "$OUT/softplus.err"; exit 1; }
python -c "import json,sys;d=json.load(open(sys.argv[1]));print('softplus',round(d['value']/1e6,2),'M/s',round(d['ms_per_step'],4),'ms',d['config']['kernels'],d['kernels_ms'])" "$OUT/softplus.json"
timeout -k 10 600 python -u -m pytest tests/test_gpu_runtime_shapes.py tests/test_gpu_generic.py tests/test_gpu_reproducibility.py \
  tests/test_gpu_agent.py tests/test_gpu_mixer.py tests/test_gpu_pipe.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; exit $rc
