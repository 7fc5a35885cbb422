#!/bin/bash
# The training-path -m gpu tests, then a config-3 A/B of one environment switch (interleaved
# on this box).  Usage: AB=RGBAC_GRAD_SINKS=0 TAG=sinks bash tools/train_check.sh
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-ab}
timeout -k 10 700 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_northstar.py tests/test_gpu_layers.py tests/test_gpu_parallel.py tests/test_gpu_models.py -x -q --timeout 200 --timeout-method thread > gpurun_out/train_check_${TAG}_tests.log 2>&1
bash tools/c3_ab.sh "${AB:?set AB}" ${TAG}
