#!/bin/bash
# config-3 A/B of one environment switch: bench --train with and without "$1" (interleaved x2)
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
T=${2:-ab}
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline > gpurun_out/c3ab_${T}_base$i.json 2> gpurun_out/c3ab_${T}_base$i.err
  env $1 timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline > gpurun_out/c3ab_${T}_var$i.json 2> gpurun_out/c3ab_${T}_var$i.err
done
