#!/bin/bash
# Run ON THE GPU BOX: a parity subset (-s: the tests print their errors and tie
# counts) then benches.   tools/r4_check.sh <tag> [pytest selection...] -> gpurun_out/<tag>/
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
SEL=${*:-tests -m gpu}
timeout -k 10 900 python -u -m pytest $SEL -x -v -s --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit 1
for algo in sequential wave sequential wave; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-companion --td-algo $algo > "$OUT/bench_$algo.json" 2> "$OUT/bench_$algo.err" \
    || { tail -5 "$OUT/bench_$algo.err"; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],round(d['value']/1e6,2),'M/s',round(d['ms_per_step'],4),'ms',d['kernels_ms'])" "$OUT/bench_$algo.json" $algo
done
