# range-count sweep of the pipelined configs[0]-shape update
set -u
OUT=gpurun_out/r5_sweep; mkdir -p $OUT
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d['value']/1e6,2),'M/s',round(d['ms_per_step'],3),'ms',d.get('kernels_ms'))" "$1"; }
B="timeout -k 10 240 python bench.py --no-cpu-baseline --no-fp32-companion"
for r in 6 8 10 12; do
  T2O_PIPELINE_RANGES=$r $B --agents 16 --batch 32 --T 150 > $OUT/c1_r$r.json 2>/dev/null || exit 1; summ $OUT/c1_r$r.json
done
for r in 8 10; do
  T2O_PIPELINE_RANGES=$r $B --agents 16 --batch 32 --T 150 > $OUT/c1b_r$r.json 2>/dev/null || exit 1; summ $OUT/c1b_r$r.json
done
$B --agents 16 --batch 128 --T 150 > $OUT/a16_b128.json 2>/dev/null || exit 1; summ $OUT/a16_b128.json
$B --agents 16 --batch 256 --T 150 --steps 8 > $OUT/a16_b256.json 2>/dev/null || exit 1; summ $OUT/a16_b256.json
$B --agents 32 --batch 64 --T 60 > $OUT/a32_b64.json 2>/dev/null || exit 1; summ $OUT/a32_b64.json
