#!/bin/bash
# PMC summary of the config-2 forward graph replay (tools/graph_trace.py): HBM traffic per
# dispatch (separate FETCH_SIZE / WRITE_SIZE passes -> tools/pmc_traffic.py, FETCH doubled per
# the gfx950 correction) and MFMA-busy per kernel (SQ_VALU_MFMA_BUSY_CYCLES pass ->
# tools/pmc_mfma.py).  GPU only.  Usage: TAG=r04_v1 bash tools/pmc_fwd.sh
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-pmc}
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_fetch -o p -- \
    python tools/graph_trace.py --reps 5 > gpurun_out/${TAG}_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_write -o p -- \
    python tools/graph_trace.py --reps 5 > gpurun_out/${TAG}_write.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVES GRBM_GUI_ACTIVE \
    --output-format csv -d gpurun_out/${TAG}_mfma -o p -- \
    python tools/graph_trace.py --reps 5 > gpurun_out/${TAG}_mfma.log 2>&1
python tools/pmc_traffic.py gpurun_out/${TAG}_fetch/p_counter_collection.csv \
    gpurun_out/${TAG}_write/p_counter_collection.csv gpurun_out/${TAG}_pmc_traffic_fwd.json 8 256
python tools/pmc_mfma.py gpurun_out/${TAG}_mfma/p_counter_collection.csv gpurun_out/${TAG}_pmc_mfma_fwd.json \
    > gpurun_out/${TAG}_pmc_mfma_fwd.txt
