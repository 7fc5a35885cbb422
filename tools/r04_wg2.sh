#!/bin/bash
# round 4: the 128 x 256 weight-gradient tile -- tests, shape timings, config-3 A/B on one box
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_northstar.py -x -q --timeout 200 --timeout-method thread -k "wgrad or train" > gpurun_out/r04_wg2_tests.log 2>&1
O=gpurun_out/r04_wgrad_times_v2.txt
: > $O
for S in "--cin 224 --cout 128 --hw 32" "--cin 96 --cout 96 --hw 64" "--cin 120 --cout 224 --hw 32" "--cin 192 --cout 192 --hw 64 --ksize 1"; do
  timeout -k 10 60 python -u tools/wgrad_probe.py $S --batch 16 --iters 30 >> $O 2>&1
  RGBAC_WGRAD_BIG=0 timeout -k 10 60 python -u tools/wgrad_probe.py $S --batch 16 --iters 30 >> $O 2>&1
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline > gpurun_out/r04_c3_big$i.json 2> gpurun_out/r04_c3_big$i.err
  RGBAC_WGRAD_BIG=0 timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline > gpurun_out/r04_c3_old$i.json 2> gpurun_out/r04_c3_old$i.err
done
