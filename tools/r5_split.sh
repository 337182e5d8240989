#!/bin/bash
# Run ON THE GPU BOX: the decoupled multi-tile mixer — its equality tests, the
# whole GPU suite, the DP tie diagnostic, then the configs it changes with the
# split forced on / off (T2O_MIXER_SPLIT) and the headline.
#   tools/r5_split.sh <tag> -> gpurun_out/<tag>/
set -u
TAG=${1:-r5_split}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ -z "${SKIP_TESTS:-}" ]; then
echo "== split tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_mixer_split.py -v -s --timeout 120 --timeout-method thread > "$OUT/split_tests.log" 2>&1
rc=$?; grep -E "passed|failed|split vs|Error|assert" "$OUT/split_tests.log" | head -30; [ $rc -ne 0 ] && exit 1
echo "== pytest"
timeout -k 10 800 python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ge 124 ] && exit 1
grep -E "FAILED|Error" "$OUT/pytest.log" | head -20
fi
echo "== diag_dp"
timeout -k 10 300 python -u tools/diag_dp_adam.py > "$OUT/diag_dp.log" 2>&1 || { tail -20 "$OUT/diag_dp.log"; exit 1; }
grep -n "resolved differently\|FFN unit\|trajectory\|cross-check\|^update" "$OUT/diag_dp.log" | head -30
echo "== benches"
B="timeout -k 10 240 python bench.py --no-cpu-baseline --no-fp32-companion"
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d['value']/1e6,2),'M/s',round(d['ms_per_step'],3),'ms',d.get('kernels_ms'))" "$1"; }
$B > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }; summ "$OUT/bench.json"
for s in 1 0; do
  T2O_MIXER_SPLIT=$s $B --agents 16 --batch 32 --T 150 > "$OUT/c1_split$s.json" 2> "$OUT/c1_split$s.err" || { tail -5 "$OUT/c1_split$s.err"; exit 1; }; summ "$OUT/c1_split$s.json"
  T2O_MIXER_SPLIT=$s $B --mode forward --agents 16 --batch 128 --T 150 > "$OUT/c2_split$s.json" 2> "$OUT/c2_split$s.err" || { tail -5 "$OUT/c2_split$s.err"; exit 1; }; summ "$OUT/c2_split$s.json"
  T2O_MIXER_SPLIT=$s $B --agents 16 --batch 1024 --T 150 --steps 5 > "$OUT/a16_split$s.json" 2> "$OUT/a16_split$s.err" || { tail -5 "$OUT/a16_split$s.err"; exit 1; }; summ "$OUT/a16_split$s.json"
  T2O_MIXER_SPLIT=$s $B --agents 64 --batch 512 --T 60 --steps 3 --warmup 1 > "$OUT/c4_split$s.json" 2> "$OUT/c4_split$s.err" || { tail -5 "$OUT/c4_split$s.err"; exit 1; }; summ "$OUT/c4_split$s.json"
done
