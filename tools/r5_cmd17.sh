# decoupled mixer at large batches: 16 AGVs x 1024, 64 AGVs x 512 (split forced vs default)
set -u
OUT=gpurun_out/r5_big; mkdir -p $OUT
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d['value']/1e6,2),'M/s',round(d['ms_per_step'],3),'ms',d['config'].get('mixer_decoupled'),d['config'].get('pipelined'),d.get('kernels_ms'))" "$1"; }
B="timeout -k 10 240 python bench.py --no-cpu-baseline --no-fp32-companion"
$B --agents 16 --batch 1024 --T 150 --steps 6 > $OUT/a16.json 2>/dev/null || exit 1; summ $OUT/a16.json
T2O_MIXER_SPLIT=1 $B --agents 16 --batch 1024 --T 150 --steps 6 > $OUT/a16_split.json 2>/dev/null || exit 1; summ $OUT/a16_split.json
T2O_MIXER_SPLIT=1 T2O_PIPELINE=0 $B --agents 16 --batch 1024 --T 150 --steps 6 > $OUT/a16_split_nopipe.json 2>/dev/null || exit 1; summ $OUT/a16_split_nopipe.json
$B --agents 64 --batch 512 --T 60 --steps 3 --warmup 2 > $OUT/a64.json 2>/dev/null || exit 1; summ $OUT/a64.json
T2O_MIXER_SPLIT=1 $B --agents 64 --batch 512 --T 60 --steps 3 --warmup 2 > $OUT/a64_split.json 2>/dev/null || exit 1; summ $OUT/a64_split.json
$B --agents 16 --batch 256 --T 150 --steps 8 > $OUT/a16_b256.json 2>/dev/null || exit 1; summ $OUT/a16_b256.json
T2O_MIXER_SPLIT=0 $B --agents 16 --batch 256 --T 150 --steps 8 > $OUT/a16_b256_nosplit.json 2>/dev/null || exit 1; summ $OUT/a16_b256_nosplit.json
