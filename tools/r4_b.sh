#!/bin/bash
# Run ON THE GPU BOX: new-path tests (launcher, paired contraction, TD loss), the
# paired vs side-stream contraction benches, then the agent-BPTT bisect A/B.
set -u
OUT=gpurun_out/r4_b
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_launch.py tests/test_gpu_reproducibility.py tests/test_gpu_td_loss.py \
  tests/test_gpu_learner.py -x -v -s --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit 1
for i in 1 2; do for m in pair side; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-companion --contract $m > "$OUT/bench_$m$i.json" 2> "$OUT/bench_$m$i.err" \
    || { tail -5 "$OUT/bench_$m$i.err"; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],round(d['value']/1e6,2),'M/s',round(d['ms_per_step'],4),'ms',d['kernels_ms'])" "$OUT/bench_$m$i.json" $m
done; done
timeout -k 10 300 python bench.py --mode loop --steps 3 --warmup 1 > "$OUT/loop.json" 2> "$OUT/loop.err" || { tail -5 "$OUT/loop.err"; exit 1; }
cut -c1-600 "$OUT/loop.json"
bash tools/ab_box.sh r4_bisect "$@"
