#!/bin/bash
# conv_pw3_kernel: parity tests, then interleaved A/B (RGBAC_PW3=0/1) of the config-4 and
# config-2 forward graphs.  GPU only.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ops.py -m gpu -k "pw3 or conv_pw_tile or stem" > gpurun_out/pw3_tests.log 2>&1
VAR=RGBAC_PW3 A=0 B=1 TAG=pw3c4 ARGS="--batch 4 --size 1024" REPS=6 bash tools/ab_env.sh
VAR=RGBAC_PW3 A=0 B=1 TAG=pw3c2 bash tools/ab_env.sh
