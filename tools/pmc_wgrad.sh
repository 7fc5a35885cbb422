#!/bin/bash
# SQ counters (two passes) of one weight-gradient shape through tools/wgrad_probe.py, the probe's
# timing, and the weight-gradient tests.  Usage: FILTER=wgrad_halo ARGS="--cin 192 --cout 192
# --hw 64 --ksize 5 --stride 2" bash tools/pmc_wgrad.sh   (GPU only; gpurun_out/pmc_wgrad.txt)
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
FILTER=${FILTER:-wgrad_halo}
ARGS=${ARGS:---cin 192 --cout 192 --hw 64 --ksize 5 --stride 2}
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/pmc_wg_a -o a -- python3 $R/tools/wgrad_probe.py $ARGS --batch 16 --iters 3 > $R/gpurun_out/pmc_wg_a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY -d $R/gpurun_out/pmc_wg_b -o b -- python3 $R/tools/wgrad_probe.py $ARGS --batch 16 --iters 3 > $R/gpurun_out/pmc_wg_b.log 2>&1
cd $R
python3 tools/pmc_db.py gpurun_out/pmc_wg_a/a_results.db --match $FILTER > gpurun_out/pmc_wgrad.txt
python3 tools/pmc_db.py gpurun_out/pmc_wg_b/b_results.db --match $FILTER >> gpurun_out/pmc_wgrad.txt
rm -rf gpurun_out/pmc_wg_a gpurun_out/pmc_wg_b
timeout -k 10 60 python -u tools/wgrad_probe.py $ARGS --batch 16 --iters 20 >> gpurun_out/pmc_wgrad.txt 2>&1
