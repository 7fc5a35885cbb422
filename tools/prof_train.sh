#!/bin/bash
# kernel trace of the config-3 training bench; one graph-replayed step's kernels summarised on
# the box (the step = the dispatches between the last two mse_bwd_kernel launches)
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
T=${1:-train}
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_$T -o t -- python3 $R/bench.py --train --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_$T.log 2>&1
cd $R
python3 tools/prof_db_stats.py gpurun_out/prof_$T/t_results.db --step-marker mse_bwd_kernel --top 70 --csv gpurun_out/prof_$T.csv > gpurun_out/prof_$T.txt
rm -rf gpurun_out/prof_$T
