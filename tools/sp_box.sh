set -e
T2O_LIB=$PWD/t2omca_amd/lib/ab_sp.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_runtime_shapes.py tests/test_gpu_generic.py -k "head or softplus or quadratic or identity or pos" > gpurun_out/sp_tests.log 2>&1
tail -2 gpurun_out/sp_tests.log
bash tools/ab_box.sh r4_sp t2omca_amd/lib/ab_base.so t2omca_amd/lib/ab_sp.so -- --qmix-pos-func softplus
