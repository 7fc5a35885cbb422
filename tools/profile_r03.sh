# Round-3 forward profile (GPU only; outputs under gpurun_out/, copied to profiles/ by hand):
#  1. rocprofv3 --kernel-trace --stats of the default bench command (no CPU baseline)
#  2. per-dispatch graph-replay trace (tools/graph_trace.py --analyze reads it)
#  3. PMC passes over the graph replay, one counter group per run:
#       HBM traffic (FETCH_SIZE, WRITE_SIZE) and MFMA utilisation
#       (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CU_CYCLES, GRBM_GUI_ACTIVE, SQ_WAVES)
# Each step has its own time limit; the first failure ends the script.
export TMPDIR=/tmp
set -e
TAG=${TAG:-r03}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o b -- python bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ktrace -o t -- python tools/graph_trace.py --reps 20 > gpurun_out/ktrace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o p -- python tools/graph_trace.py --reps 5 > gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o p -- python tools/graph_trace.py --reps 5 > gpurun_out/pmc_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_mfma -o p -- python tools/graph_trace.py --reps 5 > gpurun_out/pmc_mfma.log 2>&1
python tools/graph_trace.py --analyze gpurun_out/ktrace/t_kernel_trace.csv > gpurun_out/graph_trace.txt 2>&1 || true
python tools/pmc_mfma.py gpurun_out/pmc_mfma/p_counter_collection.csv gpurun_out/pmc_mfma.json > gpurun_out/pmc_mfma.txt 2>&1 || true
python tools/pmc_traffic.py gpurun_out/pmc_fetch/p_counter_collection.csv gpurun_out/pmc_write/p_counter_collection.csv gpurun_out/pmc_traffic.json > gpurun_out/pmc_traffic.txt 2>&1 || true
# config 4 (B=4, 1024^2): MFMA utilisation of the fused attention block where windows are many
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_mfma_c4 -o p -- python tools/graph_trace.py --reps 3 --size 1024 --batch 4 > gpurun_out/pmc_mfma_c4.log 2>&1
python tools/pmc_mfma.py gpurun_out/pmc_mfma_c4/p_counter_collection.csv gpurun_out/pmc_mfma_c4.json > gpurun_out/pmc_mfma_c4.txt 2>&1 || true
