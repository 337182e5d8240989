set -e
T2O_LIB=$PWD/t2omca_amd/lib/env_late.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_env.py tests/test_gpu_rollout.py > gpurun_out/envord_tests.log 2>&1; tail -1 gpurun_out/envord_tests.log
T2O_LIB=$PWD/t2omca_amd/lib/env_sb.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_env.py > gpurun_out/envord_tests2.log 2>&1; tail -1 gpurun_out/envord_tests2.log
bash tools/env_ab_box.sh r4_envord t2omca_amd/lib/env_base.so t2omca_amd/lib/env_sb.so t2omca_amd/lib/env_late.so
