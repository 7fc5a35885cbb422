#!/bin/bash
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_northstar.py tests/test_gpu_ops.py tests/test_gpu_layers.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_check2_tests.log 2>&1
bash tools/r04_ab_so.sh
