#!/bin/bash
# The gated last-unit-pair launch on one box (gpurun_out/r06g_*): its tests and the block /
# model tests around it, then A/B bench pairs (RGBAC_GATE_FUSED 0 / 1, alternated, forward-only
# lines) and a forward graph trace of config 2.  Stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -e
mkdir -p gpurun_out
T=${T:-r06g}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_prologue.py tests/test_gpu_northstar.py tests/test_gpu_models.py -m gpu > gpurun_out/${T}_tests.txt 2>&1
tail -n 3 gpurun_out/${T}_tests.txt
grep "gated " gpurun_out/${T}_tests.txt || true
ab() {
  for i in 1 2; do
    for v in 0 1; do
      env $1=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-parity-mode --no-dp-train --steps 50 > gpurun_out/${T}_$1_${v}_${i}.json 2>> gpurun_out/${T}_ab.err
      echo "$1=$v run $i: $(cut -c 60-200 gpurun_out/${T}_$1_${v}_${i}.json)"
    done
  done
}
ab RGBAC_GATE_FUSED
ab RGBAC_FUSED_PROLOGUE
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_tr_c2 -o t -- python tools/graph_trace.py --reps 20 > gpurun_out/${T}_tr_c2.log 2>&1
python tools/graph_trace.py --analyze gpurun_out/${T}_tr_c2/t_kernel_trace.csv > gpurun_out/${T}_tr_c2.txt
head -n 1 gpurun_out/${T}_tr_c2.txt
