set -e
export T2O_LIB=$PWD/t2omca_amd/lib/envU.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_env.py tests/test_gpu_wire.py tests/test_gpu_rollout.py tests/test_gpu_configs.py -k "env or wire or rollout or expand" > gpurun_out/envtest.log 2>&1
tail -3 gpurun_out/envtest.log
unset T2O_LIB
bash tools/env_ab_box.sh r4_env9 t2omca_amd/lib/envS.so t2omca_amd/lib/envU.so
mkdir -p gpurun_out/r4_envprof2
T2O_LIB=$PWD/t2omca_amd/lib/envProbe.so PYTHONPATH=$PWD timeout -k 10 300 python tools/env_probe.py > gpurun_out/r4_envprof2/probe.json
