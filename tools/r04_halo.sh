#!/bin/bash
# round 4: stride-1 halo weight gradient -- tests, shape timings with / without, config 3 A/B
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread -k "wgrad" > gpurun_out/r04_halo_tests.log 2>&1
O=gpurun_out/r04_halo_times.txt
: > $O
for S in "--cin 224 --cout 128 --hw 32" "--cin 96 --cout 96 --hw 64" "--cin 128 --cout 224 --hw 32"; do
  timeout -k 10 60 python -u tools/wgrad_probe.py $S --batch 16 --iters 30 >> $O 2>&1
  RGBAC_WGRAD_HALO=0 timeout -k 10 60 python -u tools/wgrad_probe.py $S --batch 16 --iters 30 >> $O 2>&1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_northstar.py tests/test_gpu_layers.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_halo_tests2.log 2>&1
bash tools/r04_c3ab.sh "RGBAC_WGRAD_HALO=0 RGBAC_WGRAD_S2=1" halo
