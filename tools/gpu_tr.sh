set -eu
OUT=gpurun_out/${1:-r2_tr}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
B="timeout -k 10 240 python bench.py --no-cpu-baseline"
$B > $OUT/bench.json 2> $OUT/bench.err
$B --agents 16 --batch 1024 --T 150 --steps 5 --no-fp32-companion > $OUT/a16.json
$B --agents 64 --batch 512 --T 60 --steps 3 --warmup 1 --no-fp32-companion > $OUT/a64.json
for f in bench a16 a64; do python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d['value']/1e6,2),round(d['ms_per_step'],3),d['kernels_ms'])" $OUT/$f.json; done
