#!/bin/bash
# Run ON THE GPU BOX: three SQ counter passes over a short serial bench, summarised per kernel.
#   tools/pmc_sq_box.sh <tag> [bench args...]   -> gpurun_out/<tag>/sq_summary.csv
set -eu
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
i=0
while read -r line; do
  case "$line" in pmc:*) ;; *) continue ;; esac
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc ${line#pmc:} --output-format csv -d "$OUT/sq$i" -o run \
    -- python3 "$R/bench.py" --no-cpu-baseline --no-fp32-companion --serial --steps 2 --warmup 1 "$@" > "$OUT/sq$i.log" 2>&1
done < "$R/profiles/pmc_sq.txt"
python3 "$R/tools/pmc_summary.py" "$OUT" "$OUT/sq_summary.csv"
