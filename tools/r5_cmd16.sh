# tape contraction on tile pairs (16x16x32): parity suite subset, A/B headline, contraction alone (serial)
set -u
OUT=gpurun_out/r5_dwp; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_learner.py tests/test_gpu_configs.py tests/test_gpu_reproducibility.py tests/test_gpu_dp_learner.py tests/test_gpu_runtime_shapes.py > $OUT/pytest.log 2>&1
rc=$?; tail -1 $OUT/pytest.log; grep FAILED $OUT/pytest.log | head; [ $rc -ne 0 ] && exit 1
AB_SERIAL= bash tools/ab_box.sh r5_dwp/head t2omca_amd/lib/ab_nopair.so t2omca_amd/lib/ab_pair.so || exit 1
bash tools/ab_box.sh r5_dwp/serial t2omca_amd/lib/ab_nopair.so t2omca_amd/lib/ab_pair.so || exit 1
