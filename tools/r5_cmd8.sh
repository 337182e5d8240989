# the block-pipelined window BPTT + lean 16-entity forward: tests, suite, configs, a trace
set -u
OUT=gpurun_out/r5_wpipe; mkdir -p $OUT gpurun_out/r5_c1prof
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d.get('config',{});print(sys.argv[1],round(d['value']/1e6,2),'M/s',round(d['ms_per_step'],3),'ms',c.get('pipelined'),d.get('kernels_ms'))" "$1"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_mixer_split.py -v -s --timeout 120 --timeout-method thread > $OUT/split_tests.log 2>&1
rc=$?; grep -E "passed|failed|vs |Error|assert" $OUT/split_tests.log | head -30; [ $rc -ne 0 ] && exit 1
timeout -k 10 800 python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -1 $OUT/pytest.log; grep -E "FAILED" $OUT/pytest.log | head; [ $rc -ne 0 ] && exit 1
B="timeout -k 10 240 python bench.py --no-cpu-baseline --no-fp32-companion"
$B --agents 16 --batch 32 --T 150 > $OUT/c1.json 2>/dev/null || exit 1; summ $OUT/c1.json
T2O_MIXS_REC=single $B --agents 16 --batch 32 --T 150 > $OUT/c1_single.json 2>/dev/null || exit 1; summ $OUT/c1_single.json
$B --agents 16 --batch 1024 --T 150 --steps 5 > $OUT/a16.json 2>/dev/null || exit 1; summ $OUT/a16.json
$B --mode forward --agents 16 --batch 128 --T 150 > $OUT/c2.json 2>/dev/null || exit 1; summ $OUT/c2.json
$B --agents 64 --batch 32 --T 60 --steps 5 > $OUT/a64_b32.json 2>/dev/null || exit 1; summ $OUT/a64_b32.json
$B > $OUT/bench.json 2>/dev/null || exit 1; summ $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5_c1prof/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-fp32-companion --agents 16 --batch 32 --T 150 --steps 6 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r5_c1prof/trace.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python3 tools/timeline_trace.py $(find gpurun_out/r5_c1prof/trace -name "*kernel_trace.csv" | head -1) adam > gpurun_out/r5_c1prof/timeline.txt
tail -3 gpurun_out/r5_c1prof/timeline.txt
