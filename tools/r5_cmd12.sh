# agent tape contraction on four FFN quarters: GPU suite, A/B old / TG2 / TG4 (headline, overlapped), a16 x 1024
set -u
OUT=gpurun_out/r5_dw; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; grep FAILED $OUT/pytest.log | head; [ $rc -ne 0 ] && exit 1
AB_SERIAL= bash tools/ab_box.sh r5_dw/head t2omca_amd/lib/ab_dwold.so t2omca_amd/lib/ab_dwtg2.so t2omca_amd/lib/ab_dwtg4.so || exit 1
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d['value']/1e6,2),'M/s',round(d['ms_per_step'],3),'ms',d.get('kernels_ms'))" "$1"; }
for v in dwold dwtg4; do
  T2O_LIB=$PWD/t2omca_amd/lib/ab_$v.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-fp32-companion --agents 16 --batch 1024 --T 150 --steps 6 > $OUT/a16_$v.json 2>/dev/null || exit 1; summ $OUT/a16_$v.json
done
