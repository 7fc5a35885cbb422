#!/bin/bash
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread -k "wgrad" > gpurun_out/r04_patch2_tests.log 2>&1
bash tools/r04_c3ab.sh "RGBAC_WGRAD_PATCH=0" patch2
