#!/bin/bash
# Round-5 evidence on one MI355X: GPU suite + DP diag + smoke (r5_check), the default
# bench line with its CPU legs, the rocprofv3 kernel trace + HBM PMC passes of the
# headline (profile_box), and the other BASELINE configs (configs_box).
#   tools/r5_final.sh <tag>   -> gpurun_out/<tag>/
set -u
TAG=${1:-r5_final}
bash tools/r5_check.sh "$TAG" || exit 1
echo "== default bench (CPU baseline legs)"
timeout -k 10 400 python bench.py > "gpurun_out/$TAG/bench_default.json" 2> "gpurun_out/$TAG/bench_default.err" || { tail -5 "gpurun_out/$TAG/bench_default.err"; exit 1; }
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(round(d['value']/1e6,2),'M/s',d['ms_per_step'],d['cpu_baseline'])" "gpurun_out/$TAG/bench_default.json"
echo "== profile"
bash tools/profile_box.sh "$TAG/prof" || exit 1
echo "== configs"
bash tools/configs_box.sh "$TAG/configs" || exit 1
echo "== SQ counters"
bash tools/pmc_sq_box.sh "$TAG/sq" || exit 1
head -8 "gpurun_out/$TAG/sq/sq_summary.csv" | cut -c1-200
