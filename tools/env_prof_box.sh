#!/bin/bash
# Run ON THE GPU BOX: env-kernel phase probe (timing-probe build) + SQ counters of a library
#   tools/env_prof_box.sh <tag> <lib.so> <probe.so>
set -eu
TAG=$1; LIB=$2; PROBE=$3
mkdir -p gpurun_out/$TAG
T2O_LIB=$PWD/$PROBE PYTHONPATH=$PWD timeout -k 10 300 python tools/env_probe.py > gpurun_out/$TAG/probe.json
T2O_LIB=$PWD/$LIB bash tools/pmc_sq_box.sh $TAG/sq --mode rollout --envs 8192 --steps 1
