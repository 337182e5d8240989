# asm bf16 conversions in the mixer TUs: parity, A/B vs the compiler's conversions, range sweep 4/5/6
set -u
OUT=gpurun_out/r5_cvt; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_mixer_split.py tests/test_gpu_mixer.py tests/test_gpu_configs.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/ab_box.sh r5_cvt/head t2omca_amd/lib/ab_cvtc.so t2omca_amd/lib/ab_cvtasm.so || exit 1
AB_SERIAL= bash tools/ab_box.sh r5_cvt/c1 t2omca_amd/lib/ab_cvtc.so t2omca_amd/lib/ab_cvtasm.so -- --agents 16 --batch 32 --T 150 || exit 1
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d['value']/1e6,2),'M/s',round(d['ms_per_step'],3),'ms',d.get('kernels_ms'))" "$1"; }
for r in 4 5 6; do
  T2O_PIPELINE_RANGES=$r timeout -k 10 240 python bench.py --no-cpu-baseline --no-fp32-companion --agents 16 --batch 32 --T 150 > $OUT/c1_r$r.json 2>/dev/null || exit 1; summ $OUT/c1_r$r.json
done
