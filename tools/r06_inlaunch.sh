#!/bin/bash
# The phase-split strided conv's slabs summed in-launch (last-arriving phase block) vs by the
# separate split-K epilogue launch (RGBAC_PATCH_INLAUNCH 1 / 0): patch-tile tests, config-2
# forward graph traces of both, alternated forward-only bench lines.  Stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -e
mkdir -p gpurun_out
T=${T:-r06k}
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_northstar.py tests/test_gpu_models.py -m gpu > gpurun_out/${T}_tests.txt 2>&1
tail -n 1 gpurun_out/${T}_tests.txt
for v in 0 1; do
  RGBAC_PATCH_INLAUNCH=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_tr_$v -o t -- python tools/graph_trace.py --reps 20 > gpurun_out/${T}_tr_$v.log 2>&1
  python tools/graph_trace.py --analyze gpurun_out/${T}_tr_$v/t_kernel_trace.csv > gpurun_out/${T}_tr_$v.txt
  echo "inlaunch=$v: $(head -n 1 gpurun_out/${T}_tr_$v.txt)"
  sed -n 9,12p gpurun_out/${T}_tr_$v.txt
done
for i in 1 2 3; do
  for v in 0 1; do
    RGBAC_PATCH_INLAUNCH=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-parity-mode --no-dp-train --steps 50 > gpurun_out/${T}_ab_${v}_${i}.json 2>> gpurun_out/${T}_ab.err
    echo "inlaunch=$v run $i: $(cut -c 100-150 gpurun_out/${T}_ab_${v}_${i}.json)"
  done
done
