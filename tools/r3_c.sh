#!/bin/bash
# Run ON THE GPU BOX: new GPU tests, the dp2 gloo rehearsal, the rollout profile
# (kernel trace + HBM PMC passes) and the default bench lines (train + rollout).
set -eu
OUT=gpurun_out/r3_c
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "abi_mixer or rccl or obsbranch or dp_learner or rollout" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/r3_dp_rehearsal.sh r3_c
bash tools/profile_box.sh r3_c/roll --mode rollout --steps 4 --warmup 1
cat $OUT/roll/kernel_stats.csv | head -12
timeout -k 10 300 python bench.py --mode rollout > $OUT/rollout.json 2> $OUT/rollout.err || { tail $OUT/rollout.err; exit 1; }
cat $OUT/rollout.json
timeout -k 10 300 python bench.py --mode rollout --compact-obs --no-cpu-baseline > $OUT/rollout_wire.json 2> $OUT/rollout_wire.err || { tail $OUT/rollout_wire.err; exit 1; }
cat $OUT/rollout_wire.json
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
