#!/bin/bash
# the full -m gpu suite, then the library A/B against the previous commit's build
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_gputest.log 2>&1
bash tools/r04_ab_so.sh
RGBAC_WGRAD_TARGET_BIG=128 timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline --no-dp-train > gpurun_out/ab_c3_tb128.json 2> gpurun_out/ab_c3_tb128.err
RGBAC_WGRAD_TARGET=512 timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline --no-dp-train > gpurun_out/ab_c3_t512.json 2> gpurun_out/ab_c3_t512.err
RGBAC_WGRAD_TARGET=2048 timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline --no-dp-train > gpurun_out/ab_c3_t2048.json 2> gpurun_out/ab_c3_t2048.err
timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline --no-dp-train > gpurun_out/ab_c3_def2.json 2> gpurun_out/ab_c3_def2.err
