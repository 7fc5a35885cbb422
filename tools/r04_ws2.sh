#!/bin/bash
# round 4: polyphase 5x5/s2 weight gradient -- tests, shape timings with / without, config 3
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread -k "wgrad" > gpurun_out/r04_ws2_tests.log 2>&1
O=gpurun_out/r04_ws2_times.txt
: > $O
for S in "--cin 192 --cout 192 --hw 64" "--cin 192 --cout 192 --hw 32"; do
  timeout -k 10 60 python -u tools/wgrad_probe.py $S --ksize 5 --stride 2 --batch 16 --iters 20 >> $O 2>&1
  RGBAC_WGRAD_S2=0 timeout -k 10 60 python -u tools/wgrad_probe.py $S --ksize 5 --stride 2 --batch 16 --iters 20 >> $O 2>&1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_northstar.py tests/test_gpu_layers.py tests/test_gpu_fused.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_ws2_tests2.log 2>&1
timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline > gpurun_out/r04_c3_ws2.json 2> gpurun_out/r04_c3_ws2.err
RGBAC_WGRAD_S2=0 timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline > gpurun_out/r04_c3_nows2.json 2> gpurun_out/r04_c3_nows2.err
