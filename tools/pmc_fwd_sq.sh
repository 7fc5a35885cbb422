#!/bin/bash
# SQ instruction / wait counters (two passes) of every kernel in the config-2 forward graph
# replay (tools/graph_trace.py).  GPU only; gpurun_out/${TAG}_pmc_sq.txt
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
TAG=${TAG:-fwd}
ARGS=${ARGS:---reps 3}
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/pmc_sq_a -o a -- python3 $R/tools/graph_trace.py $ARGS > $R/gpurun_out/pmc_sq_a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY -d $R/gpurun_out/pmc_sq_b -o b -- python3 $R/tools/graph_trace.py $ARGS > $R/gpurun_out/pmc_sq_b.log 2>&1
cd $R
python3 tools/pmc_db.py gpurun_out/pmc_sq_a/a_results.db > gpurun_out/${TAG}_pmc_sq.txt
python3 tools/pmc_db.py gpurun_out/pmc_sq_b/b_results.db >> gpurun_out/${TAG}_pmc_sq.txt
rm -rf gpurun_out/pmc_sq_a gpurun_out/pmc_sq_b
