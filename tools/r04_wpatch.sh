#!/bin/bash
# round 4: the patch weight-gradient kernel (narrow-output 3x3 convs) -- tests, shape timings
# with / without it, config 3, the forward A/B against the previous commit's build, and a
# kernel-stats profile of the training step
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread -k "wgrad" > gpurun_out/r04_wpatch_tests.log 2>&1
O=gpurun_out/r04_wpatch_times.txt
: > $O
for S in "--cin 32 --cout 32 --hw 256" "--cin 128 --cout 8 --hw 32"; do
  timeout -k 10 60 python -u tools/wgrad_probe.py $S --batch 16 --iters 30 >> $O 2>&1
  RGBAC_WGRAD_PATCH=0 timeout -k 10 60 python -u tools/wgrad_probe.py $S --batch 16 --iters 30 >> $O 2>&1
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_northstar.py tests/test_gpu_layers.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_wpatch_tests2.log 2>&1
timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline > gpurun_out/r04_c3_wpatch.json 2> gpurun_out/r04_c3_wpatch.err
RGBAC_WGRAD_PATCH=0 timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline > gpurun_out/r04_c3_nowpatch.json 2> gpurun_out/r04_c3_nowpatch.err
bash tools/r04_ab_so.sh
