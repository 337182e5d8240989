# Run ON THE GPU BOX: mixer parity tests on the candidate build, then the parity-gated headline A/B
set -e
T2O_LIB=$PWD/t2omca_amd/lib/ab_elu.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mixer.py tests/test_gpu_runtime_shapes.py tests/test_gpu_configs.py tests/test_gpu_learner.py tests/test_gpu_generic.py > gpurun_out/elu_tests.log 2>&1
tail -1 gpurun_out/elu_tests.log
bash tools/ab_box.sh r4_elu t2omca_amd/lib/ab_base.so t2omca_amd/lib/ab_elu.so
