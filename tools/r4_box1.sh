set -e
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rollout.py tests/test_gpu_env.py > gpurun_out/rollout_tests.log 2>&1
tail -2 gpurun_out/rollout_tests.log
timeout -k 10 200 python bench.py --mode rollout --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/rollout_fp32.json
timeout -k 10 200 python bench.py --mode rollout --steps 5 --warmup 2 --no-cpu-baseline --rollout-precision bf16 > gpurun_out/rollout_bf16.json
python -c "
import json
for f in ('fp32','bf16'):
    d=json.load(open(f'gpurun_out/rollout_{f}.json')); print(f, round(d['value']/1e6,1), d['kernels_ms'], round(d['per_env_step_ms'],4))"
bash tools/env_prof_box.sh r4_envprof t2omca_amd/lib/libt2omca.so t2omca_amd/lib/envProbe.so
