#!/bin/bash
# Run ON THE GPU BOX: the GPU suite, the default bench line (with its CPU legs),
# the rollout line (configs[4] defaults) and one SQ counter pass (LDS bank
# conflicts) over the serial train bench.
set -eu
TAG=${1:-r3_d}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cat /sys/fs/cgroup/cpu.max > $OUT/host_cpus.txt 2>&1 || true
python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'OMP', os.environ.get('OMP_NUM_THREADS'))" >> $OUT/host_cpus.txt
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 \
  || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cut -c1-1500 $OUT/bench.json
timeout -k 10 300 python bench.py --mode rollout > $OUT/rollout.json 2> $OUT/rollout.err || { tail $OUT/rollout.err; exit 1; }
cut -c1-1500 $OUT/rollout.json
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_FLAT \
  --output-format csv -d $R/$OUT/sq2 -o run -- python3 $R/bench.py --no-cpu-baseline --no-fp32-companion --serial --steps 2 --warmup 1 > $R/$OUT/sq2.log 2>&1
cd $R
python3 tools/pmc_summary.py $OUT $OUT/sq_summary.csv > /dev/null
cat $OUT/sq_summary.csv | cut -c1-300
