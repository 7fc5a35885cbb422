#!/bin/bash
# ws-8 window block inside the config-4 forward graph: the round-3 kernel (RGBAC_WINBLOCK_FORM=2)
# against the head-pair kernels (=3), two alternations, rocprofv3 kernel trace -> per-dispatch
# tables gpurun_out/${TAG}_f{2,3}_{1,2}.txt.  GPU only.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-wbab}
for r in 1 2; do
  for f in 2 3; do
    RGBAC_WINBLOCK_FORM=$f timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
        -d gpurun_out/${TAG}_f${f}_$r -o t -- python tools/graph_trace.py --reps 6 --batch 4 --size 1024 \
        > gpurun_out/${TAG}_f${f}_$r.log 2>&1
    python tools/graph_trace.py --analyze gpurun_out/${TAG}_f${f}_$r/t_kernel_trace.csv > gpurun_out/${TAG}_f${f}_$r.txt
    rm -rf gpurun_out/${TAG}_f${f}_$r
  done
done
