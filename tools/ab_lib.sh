#!/bin/bash
# A/B of two library builds on one box: the working tree's librgbac_hip.so against
# rgbac/librgbac_hip_prev.so, interleaved; config 3 (with per-layer tables) and config 2.
# Usage: TAG=x TESTS="tests/test_gpu_ops.py -k spatial" bash tools/ab_lib.sh
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
P=deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd/rgbac/librgbac_hip_prev.so
T=${TAG:-ab}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_${T}_tests.log 2>&1
fi
for i in 1 2; do
  L1=""; L2=""
  if [ $i = 2 ]; then L1="--layers gpurun_out/ab_${T}_c3_new_layers.txt"; L2="--layers gpurun_out/ab_${T}_c3_old_layers.txt"; fi
  timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline $L1 > gpurun_out/ab_${T}_c3_new$i.json 2> gpurun_out/ab_${T}_c3_new$i.err
  RGBAC_LIB_PATH=$P timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline $L2 > gpurun_out/ab_${T}_c3_old$i.json 2> gpurun_out/ab_${T}_c3_old$i.err
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --no-dp-train > gpurun_out/ab_${T}_c2_new$i.json 2> gpurun_out/ab_${T}_c2_new$i.err
  RGBAC_LIB_PATH=$P timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --no-dp-train > gpurun_out/ab_${T}_c2_old$i.json 2> gpurun_out/ab_${T}_c2_old$i.err
done
