# A=16 forward at two waves per SIMD (ab_ag16lean) vs base on the A=16 shapes; a
# kernel trace of the pipelined configs[0]-shape update
set -u
OUT=gpurun_out/r5_ag16; mkdir -p $OUT
for lib in ab_base ab_ag16lean; do
  for i in 1 2; do
    T2O_LIB=$PWD/t2omca_amd/lib/$lib.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-fp32-companion --agents 16 --batch 1024 --T 150 --steps 5 > $OUT/${lib}_a16_$i.json 2>/dev/null || exit 1
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d['ms_per_step'],3),d['kernels_ms'])" $OUT/${lib}_a16_$i.json
  done
done
T2O_LIB=$PWD/t2omca_amd/lib/ab_ag16lean.so timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_runtime_shapes.py -x -q --timeout 120 --timeout-method thread > $OUT/ag16lean_parity.log 2>&1; tail -1 $OUT/ag16lean_parity.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5_c1prof/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-fp32-companion --agents 16 --batch 32 --T 150 --steps 6 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r5_c1prof/trace.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python3 tools/timeline_trace.py $(find gpurun_out/r5_c1prof/trace -name "*kernel_trace.csv" | head -1) adam > gpurun_out/r5_c1prof/timeline.txt
tail -5 gpurun_out/r5_c1prof/timeline.txt
