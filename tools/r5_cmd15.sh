# A/B: HEAD vs key-tile mask + bf16 ReLU (rbf) vs key-tile mask + fp32 ReLU (rf32); parity gate in ab_box
set -u
AB_SERIAL= bash tools/ab_box.sh r5_relu/head t2omca_amd/lib/ab_head.so t2omca_amd/lib/ab_rbf.so t2omca_amd/lib/ab_rf32.so || exit 1
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mixer_split.py tests/test_gpu_mixer.py tests/test_gpu_agent.py > gpurun_out/r5_relu/pytest.log 2>&1; tail -1 gpurun_out/r5_relu/pytest.log
