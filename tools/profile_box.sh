#!/bin/bash
# Run ON THE GPU BOX (via gpurun) from the repo root: kernel-trace stats of the
# default bench workload plus the two HBM-traffic PMC passes (FETCH_SIZE and
# WRITE_SIZE do not fit one TCC pass), summarised into gpurun_out/<tag>/.
#   tools/profile_box.sh <tag> [bench args...]
set -eu
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 "$R/bench.py" --no-cpu-baseline --no-fp32-companion "$@" > "$OUT/trace.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run \
  -- python3 "$R/bench.py" --no-cpu-baseline --no-fp32-companion --steps 3 --warmup 1 "$@" > "$OUT/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run \
  -- python3 "$R/bench.py" --no-cpu-baseline --no-fp32-companion --steps 3 --warmup 1 "$@" > "$OUT/write.log" 2>&1
python3 "$R/tools/pmc_traffic.py" "$OUT/fetch" "$OUT/write" "$OUT/hbm_traffic.json" \
  "$(python3 "$R/bench.py" --print-workload-tag "$@")" > /dev/null
find "$OUT/trace" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
tail -1 "$OUT/trace.log" > "$OUT/bench.json" || true
echo "profile $TAG done"
