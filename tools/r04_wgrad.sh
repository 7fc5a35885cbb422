#!/bin/bash
# wgrad diagnostics (round 4): timings of the main training weight-gradient shapes, then PMC
# counter groups over one of them.  GPU only; outputs under gpurun_out/.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
O=gpurun_out/r04_wgrad_times.txt
: > $O
for S in "--cin 224 --cout 128 --hw 32" "--cin 96 --cout 96 --hw 64" "--cin 192 --cout 96 --hw 64 --ksize 1" \
         "--cin 120 --cout 224 --hw 32" "--cin 32 --cout 32 --hw 256" "--cin 192 --cout 192 --hw 64 --ksize 1"; do
  timeout -k 10 60 python -u tools/wgrad_probe.py $S --batch 16 --iters 30 >> $O 2>&1
done
bash tools/pmc_kernel.sh wg wgrad_ring python tools/wgrad_probe.py --cin 224 --cout 128 --hw 32 --batch 16 --iters 10 > gpurun_out/r04_wgrad_pmc.txt 2>&1
