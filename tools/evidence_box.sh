#!/bin/bash
# A round's evidence on one MI355X (run ON THE GPU BOX):   tools/evidence_box.sh <tag> [parts]
#   check    GPU suite (-v -s: the parity tests print their errors and ReLU-tie
#            reports), the DP tie diagnostic, smoke, the bench line without CPU legs
#   bench    the default bench line with its CPU baseline legs
#   prof     rocprofv3 kernel trace + HBM PMC passes of the headline (profile_box.sh)
#   configs  the other BASELINE configs (configs_box.sh)
#   sq       SQ counters (pmc_sq_box.sh)
# parts default: "check bench prof configs sq".  Output: gpurun_out/<tag>/.
# Every step is bounded; a failing or timed-out GPU step ends the script.
set -u
TAG=${1:-evidence}
PARTS=${2:-check bench prof configs sq}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for part in $PARTS; do
  case $part in
    check)
      echo "== pytest"
      timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
        > "$OUT/pytest.log" 2>&1
      rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -gt 1 ] && exit 1
      echo "== diag_dp"
      timeout -k 10 300 python -u tools/diag_dp_adam.py > "$OUT/diag_dp.log" 2>&1 || { tail -20 "$OUT/diag_dp.log"; exit 1; }
      grep -n "update\|resolved differently\|FFN unit\|trajectory\|cross-check" "$OUT/diag_dp.log" | head -20
      echo "== smoke"
      timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
      tail -1 "$OUT/smoke.log"
      echo "== bench (no CPU legs)"
      timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
      python -c "import json,sys;d=json.load(open(sys.argv[1]));print(round(d['value']/1e6,2),'M/s',round(d['ms_per_step'],3),'ms',d['kernels_ms'],d['roofline']['kernel'],round(d['roofline']['frac'],4))" "$OUT/bench.json"
      ;;
    bench)
      echo "== default bench (CPU baseline legs)"
      timeout -k 10 400 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail -5 "$OUT/bench_default.err"; exit 1; }
      python -c "import json,sys;d=json.load(open(sys.argv[1]));print(round(d['value']/1e6,2),'M/s',d['ms_per_step'],d['cpu_baseline'])" "$OUT/bench_default.json"
      ;;
    prof) echo "== profile"; bash tools/profile_box.sh "$TAG/prof" || exit 1 ;;
    configs) echo "== configs"; bash tools/configs_box.sh "$TAG/configs" || exit 1 ;;
    sq)
      echo "== SQ counters"; bash tools/pmc_sq_box.sh "$TAG/sq" || exit 1
      head -8 "gpurun_out/$TAG/sq/sq_summary.csv" | cut -c1-200 ;;
    *) echo "unknown part $part"; exit 2 ;;
  esac
done
exit 0
