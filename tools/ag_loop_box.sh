# Run ON THE GPU BOX: rollout agent-step A/B (fp32 and bf16) of two builds + headline train A/B
set -e
mkdir -p gpurun_out/r4_agloop
for i in 1 2; do
  for lib in envBase agLoop2; do
    for p in fp32 bf16; do
      T2O_LIB=$PWD/t2omca_amd/lib/$lib.so timeout -k 10 200 python bench.py --mode rollout --steps 3 --warmup 1 --no-cpu-baseline --kernel-timer-every 1 --rollout-precision $p > gpurun_out/r4_agloop/${lib}_${p}_$i.json
      python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],d['kernels_ms'])" gpurun_out/r4_agloop/${lib}_${p}_$i.json
    done
  done
done
T2O_LIB=$PWD/t2omca_amd/lib/agLoop2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rollout.py tests/test_gpu_agent.py > gpurun_out/r4_agloop/tests.log 2>&1; tail -1 gpurun_out/r4_agloop/tests.log
bash tools/ab_box.sh r4_agloop_train t2omca_amd/lib/ab_base.so t2omca_amd/lib/agLoop2.so
