#!/bin/bash
# round 4: activation backward folded into the consumer's input-gradient conv (DGELU / DLRELU)
# -- training-path tests, then a config-3 A/B (RGBAC_DEFER_ACT=0 = separate act_bwd passes)
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_northstar.py tests/test_gpu_layers.py tests/test_gpu_parallel.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_defer_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline > gpurun_out/r04_c3_defer$i.json 2> gpurun_out/r04_c3_defer$i.err
  RGBAC_DEFER_ACT=0 timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline > gpurun_out/r04_c3_nodefer$i.json 2> gpurun_out/r04_c3_nodefer$i.err
done
timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline > gpurun_out/r04_c2_defer.json 2> gpurun_out/r04_c2_defer.err
