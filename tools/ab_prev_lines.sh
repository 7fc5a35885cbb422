#!/bin/bash
# A/B of two library builds on one box: the working tree's librgbac_hip.so against
# rgbac/librgbac_hip_prev.so (a build of the previous commit), interleaved
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
P=deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd/rgbac/librgbac_hip_prev.so
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline > gpurun_out/ab_c2_new$i.json 2> gpurun_out/ab_c2_new$i.err
  RGBAC_DEFER_ACT=0 RGBAC_WGRAD_PATCH=0 RGBAC_LIB_PATH=$P timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline > gpurun_out/ab_c2_old$i.json 2> gpurun_out/ab_c2_old$i.err
done
timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline --layers gpurun_out/ab_c3_new_layers.txt > gpurun_out/ab_c3_new.json 2> gpurun_out/ab_c3_new.err
RGBAC_DEFER_ACT=0 RGBAC_WGRAD_PATCH=0 RGBAC_LIB_PATH=$P timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline > gpurun_out/ab_c3_old.json 2> gpurun_out/ab_c3_old.err
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c3 -o c3 -- python3 $GRAFT_REPO_ROOT/bench.py --train --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_c3.log 2>&1
