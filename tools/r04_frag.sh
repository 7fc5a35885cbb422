#!/bin/bash
# round 4: fragment-major training packs -- training tests, then re-tune + A/B of the cache
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_northstar.py tests/test_gpu_layers.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_frag_tests.log 2>&1
bash tools/retune_train.sh
