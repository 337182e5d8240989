# Run ON THE GPU BOX: env parity tests on a candidate env build, then an interleaved rollout A/B
#   tools/env_test_box.sh <tag> <candidate.so> <baseline.so>
set -e
TAG=$1; CAND=$2; BASE=$3
mkdir -p gpurun_out/$TAG
T2O_LIB=$PWD/$CAND timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_env.py tests/test_gpu_wire.py tests/test_gpu_rollout.py tests/test_gpu_configs.py -k "env or wire or rollout or expand" > gpurun_out/$TAG/envtest.log 2>&1
tail -1 gpurun_out/$TAG/envtest.log
bash tools/env_ab_box.sh $TAG $BASE $CAND
