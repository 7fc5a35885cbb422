#!/bin/bash
# forward A/B of the working tree's library against rgbac/librgbac_hip_prev.so on one box:
# two interleaved bench runs each, the second pair with per-layer tables
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
P=deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd/rgbac/librgbac_hip_prev.so
T=${1:-x}
for i in 1 2; do
  L1=""; L2=""
  if [ $i = 2 ]; then L1="--layers gpurun_out/abf_${T}_new_layers.txt"; L2="--layers gpurun_out/abf_${T}_old_layers.txt"; fi
  timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --no-dp-train $L1 > gpurun_out/abf_${T}_new$i.json 2> gpurun_out/abf_${T}_new$i.err
  RGBAC_DEFER_ACT=0 RGBAC_WGRAD_PATCH=0 RGBAC_LIB_PATH=$P timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --no-dp-train $L2 > gpurun_out/abf_${T}_old$i.json 2> gpurun_out/abf_${T}_old$i.err
done
