set -e
export T2O_LIB=$PWD/t2omca_amd/lib/envQ.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_env.py tests/test_gpu_wire.py tests/test_gpu_rollout.py tests/test_gpu_configs.py -k "env or wire or rollout or expand" > gpurun_out/envtest.log 2>&1
tail -3 gpurun_out/envtest.log
unset T2O_LIB
bash tools/env_ab_box.sh r4_env6 t2omca_amd/lib/envA.so t2omca_amd/lib/envM.so t2omca_amd/lib/envQ.so
