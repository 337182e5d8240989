#!/bin/bash
# Run ON THE GPU BOX: one SQ counter pass (LDS instructions / bank conflicts / VALU)
# per library build over a short serial bench; per-kernel summaries.
#   tools/r3_pmc_ab.sh <tag> <lib.so>...
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp
export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename "$lib" .so)
  OUT=$R/gpurun_out/$TAG/$n
  mkdir -p "$OUT"
  T2O_LIB=$R/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS \
    SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_FLAT \
    --output-format csv -d "$OUT/sq" -o run \
    -- python3 "$R/bench.py" --no-cpu-baseline --no-fp32-companion --serial --steps 2 --warmup 1 > "$OUT/sq.log" 2>&1 \
    || { tail -5 "$OUT/sq.log"; exit 1; }
  T2O_LIB=$R/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS \
    --output-format csv -d "$OUT/sq2" -o run \
    -- python3 "$R/bench.py" --no-cpu-baseline --no-fp32-companion --serial --steps 2 --warmup 1 > "$OUT/sq2.log" 2>&1 \
    || { tail -5 "$OUT/sq2.log"; exit 1; }
  python3 "$R/tools/pmc_summary.py" "$OUT" "$OUT/sq_summary.csv" > /dev/null
  echo "== $n"; cut -c1-400 "$OUT/sq_summary.csv"
done
