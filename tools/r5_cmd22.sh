# final-state check: GPU suite, smoke, default bench; 32-AGV shapes for the DESIGN table
set -u
OUT=gpurun_out/r5_last; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -q -s --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -1 $OUT/pytest.log; grep -A3 "differing indices\|^FAILED" $OUT/pytest.log | head -10; [ $rc -ne 0 ] && exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d['value']/1e6,2),'M/s',round(d['ms_per_step'],3),'ms',d.get('kernels_ms'))" "$1"; }
summ $OUT/bench.json
timeout -k 10 240 python bench.py --no-cpu-baseline --no-fp32-companion --agents 32 --batch 1024 --T 60 --steps 4 --warmup 2 > $OUT/a32.json 2>/dev/null || exit 1; summ $OUT/a32.json
timeout -k 10 240 python bench.py --no-cpu-baseline --no-fp32-companion --agents 12 --batch 1024 --T 60 --steps 8 > $OUT/a12.json 2>/dev/null || exit 1; summ $OUT/a12.json
