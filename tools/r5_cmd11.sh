# scattered agent softmax: GPU suite, smoke, headline bench, configs[0]-shape bench
set -u
bash tools/r5_check.sh r5_rs || exit 1
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d['value']/1e6,2),'M/s',round(d['ms_per_step'],3),'ms',d.get('kernels_ms'))" "$1"; }
B="timeout -k 10 240 python bench.py --no-cpu-baseline --no-fp32-companion"
for r in 6 10; do
  T2O_PIPELINE_RANGES=$r $B --agents 16 --batch 32 --T 150 > gpurun_out/r5_rs/c1_r$r.json 2>/dev/null || exit 1; summ gpurun_out/r5_rs/c1_r$r.json
done
$B --agents 16 --batch 1024 --T 150 --steps 8 > gpurun_out/r5_rs/a16_b1024.json 2>/dev/null || exit 1; summ gpurun_out/r5_rs/a16_b1024.json
