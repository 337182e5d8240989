#!/bin/bash
# Run ON THE GPU BOX: GPU suite (-v -s: the parity tests print their errors and
# ReLU-tie reports), the DP tie diagnostic, smoke, and the default bench line
# without its CPU legs.   tools/r5_check.sh <tag> [pytest-args...] -> gpurun_out/<tag>/
set -u
TAG=${1:-r5_check}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
echo "== pytest"
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread "$@" > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ge 124 ] && exit 1
echo "== diag_dp"
timeout -k 10 300 python -u tools/diag_dp_adam.py > "$OUT/diag_dp.log" 2>&1 || { tail -20 "$OUT/diag_dp.log"; exit 1; }
grep -n "update\|resolved differently\|FFN unit\|trajectory\|cross-check" "$OUT/diag_dp.log" | head -40
echo "== smoke"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
echo "== bench"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(round(d['value']/1e6,2),'M/s',round(d['ms_per_step'],3),'ms',d['kernels_ms'],d['roofline']['kernel'],round(d['roofline']['frac'],4))" "$OUT/bench.json"
exit $rc
