# paired 16x16x32 key products (packed bf16 conversions), bias-in-accumulator, packed ReLU:
# GPU suite, A/B base / new at the headline (overlapped), configs[0]-shape
set -u
OUT=gpurun_out/r5_kp; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; grep FAILED $OUT/pytest.log | head; [ $rc -ne 0 ] && exit 1
AB_SERIAL= bash tools/ab_box.sh r5_kp/head t2omca_amd/lib/ab_base.so t2omca_amd/lib/ab_new.so || exit 1
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d['value']/1e6,2),'M/s',round(d['ms_per_step'],3),'ms',d.get('kernels_ms'))" "$1"; }
for v in base new; do
  T2O_LIB=$PWD/t2omca_amd/lib/ab_$v.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-fp32-companion --agents 16 --batch 32 --T 150 > $OUT/c1_$v.json 2>/dev/null || exit 1; summ $OUT/c1_$v.json
done
