# HBM traffic per dispatch of the config-4 forward (B=4, 1024x1024) graph replay: separate
# FETCH_SIZE / WRITE_SIZE passes -> tools/pmc_traffic.py.  GPU only.
export TMPDIR=/tmp
set -e
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmcb_$C -o p -- \
      python tools/graph_trace.py --batch 4 --size 1024 --reps 3 > gpurun_out/pmcb_$C.log 2>&1
done
python tools/pmc_traffic.py gpurun_out/pmcb_FETCH_SIZE/p_counter_collection.csv \
    gpurun_out/pmcb_WRITE_SIZE/p_counter_collection.csv gpurun_out/pmc_traffic_fwd_b4_1024.json 4 1024 \
    > gpurun_out/pmc_traffic_fwd_b4_1024.txt
rm -rf gpurun_out/pmcb_FETCH_SIZE gpurun_out/pmcb_WRITE_SIZE
