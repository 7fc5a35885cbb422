#!/bin/bash
# MFMA-busy per kernel of the config-4 forward (B=4, 1024x1024) graph replay: one
# SQ_VALU_MFMA_BUSY_CYCLES pass -> tools/pmc_mfma.py.  GPU only.  Usage: TAG=r06 bash tools/pmc_mfma_c4.sh
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-pmc}
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVES GRBM_GUI_ACTIVE \
    --output-format csv -d gpurun_out/${TAG}_mfma_c4 -o p -- \
    python tools/graph_trace.py --batch 4 --size 1024 --reps 3 > gpurun_out/${TAG}_mfma_c4.log 2>&1
python tools/pmc_mfma.py gpurun_out/${TAG}_mfma_c4/p_counter_collection.csv gpurun_out/${TAG}_pmc_mfma_c4.json \
    > gpurun_out/${TAG}_pmc_mfma_c4.txt
rm -rf gpurun_out/${TAG}_mfma_c4
