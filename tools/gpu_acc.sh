set -eu
OUT=gpurun_out/${1:-r2_acc}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 240 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(round(d['value']/1e6,2),round(d['ms_per_step'],3),d['kernels_ms'])" $OUT/bench.json
bash tools/ab_box.sh ${1:-r2_acc}_ab t2omca_amd/lib/ab_sw.so t2omca_amd/lib/ab_acc.so
