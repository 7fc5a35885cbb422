#!/bin/bash
# Full -m gpu suite + smoke, then A/B pairs of the gated last unit pair (forward-only lines,
# alternated) and a config-2 forward graph trace (gpurun_out/${T}_*).  Stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -e
mkdir -p gpurun_out
T=${T:-r06i}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1
tail -n 2 gpurun_out/${T}_gputest.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1
tail -n 2 gpurun_out/${T}_smoke.txt
for i in 1 2 3; do
  for v in 0 1; do
    RGBAC_GATE_FUSED=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-parity-mode --no-dp-train --steps 50 > gpurun_out/${T}_gate_${v}_${i}.json 2>> gpurun_out/${T}_ab.err
    echo "RGBAC_GATE_FUSED=$v run $i: $(cut -c 100-190 gpurun_out/${T}_gate_${v}_${i}.json)"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_tr_c2 -o t -- python tools/graph_trace.py --reps 20 > gpurun_out/${T}_tr_c2.log 2>&1
python tools/graph_trace.py --analyze gpurun_out/${T}_tr_c2/t_kernel_trace.csv > gpurun_out/${T}_tr_c2.txt
head -n 1 gpurun_out/${T}_tr_c2.txt
grep "ru_stream\|prologue\|mse_\|finalize" gpurun_out/${T}_tr_c2.txt | head -12
