#!/bin/bash
# Run ON THE GPU BOX: the pipelined small-batch update — split/pipeline tests, the
# GPU suite, configs[0]-shape / configs[1] / headline benches, a range-count sweep.
#   tools/r5_pipe.sh <tag> -> gpurun_out/<tag>/
set -u
TAG=${1:-r5_pipe}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d.get('config',{});print(sys.argv[1],round(d['value']/1e6,2),'M/s',round(d['ms_per_step'],3),'ms',c.get('pipelined'),c.get('mixer_decoupled'),d.get('kernels_ms'))" "$1"; }
echo "== split/pipeline tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_mixer_split.py -v -s --timeout 120 --timeout-method thread > "$OUT/split_tests.log" 2>&1
rc=$?; grep -E "passed|failed|vs |Error|assert" "$OUT/split_tests.log" | head -30; [ $rc -ne 0 ] && exit 1
if [ -z "${SKIP_SUITE:-}" ]; then
echo "== pytest"
timeout -k 10 800 python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -1 "$OUT/pytest.log"; [ $rc -ge 124 ] && exit 1
grep -E "FAILED|Error" "$OUT/pytest.log" | head -20
fi
echo "== benches"
B="timeout -k 10 240 python bench.py --no-cpu-baseline --no-fp32-companion"
$B --agents 16 --batch 32 --T 150 > "$OUT/c1.json" 2> "$OUT/c1.err" || { tail -5 "$OUT/c1.err"; exit 1; }; summ "$OUT/c1.json"
for r in 5 15 25; do
  T2O_PIPELINE_RANGES=$r $B --agents 16 --batch 32 --T 150 > "$OUT/c1_r$r.json" 2> "$OUT/c1_r$r.err" || { tail -5 "$OUT/c1_r$r.err"; exit 1; }; summ "$OUT/c1_r$r.json"
done
T2O_PIPELINE=0 $B --agents 16 --batch 32 --T 150 > "$OUT/c1_nopipe.json" 2> "$OUT/c1_nopipe.err" || { tail -5 "$OUT/c1_nopipe.err"; exit 1; }; summ "$OUT/c1_nopipe.json"
$B --agents 16 --batch 128 --T 150 > "$OUT/a16_b128.json" 2> "$OUT/a16_b128.err" || { tail -5 "$OUT/a16_b128.err"; exit 1; }; summ "$OUT/a16_b128.json"
$B --agents 16 --batch 256 --T 150 --steps 8 > "$OUT/a16_b256.json" 2> "$OUT/a16_b256.err" || { tail -5 "$OUT/a16_b256.err"; exit 1; }; summ "$OUT/a16_b256.json"
$B --mode forward --agents 16 --batch 128 --T 150 > "$OUT/c2.json" 2> "$OUT/c2.err" || { tail -5 "$OUT/c2.err"; exit 1; }; summ "$OUT/c2.json"
$B > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }; summ "$OUT/bench.json"
