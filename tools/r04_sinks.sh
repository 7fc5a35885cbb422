#!/bin/bash
# round 4: activation-gradient sinks -- training tests, then config-3 A/B (RGBAC_GRAD_SINKS=0)
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_northstar.py tests/test_gpu_layers.py tests/test_gpu_parallel.py tests/test_gpu_models.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_sinks_tests.log 2>&1
bash tools/r04_c3ab.sh "${AB:-RGBAC_GRAD_SINKS=0}" ${TAG:-sinks}
