#!/bin/bash
# Round-5 closing profile of the default bench command (config 2): rocprofv3 kernel-trace stats
# of that command, the PMC HBM traffic per kernel (separate FETCH_SIZE / WRITE_SIZE passes over
# the forward graph replay), then the bench line reading that traffic summary.  GPU only.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o b -- python bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o p -- python tools/graph_trace.py --reps 5 > gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o p -- python tools/graph_trace.py --reps 5 > gpurun_out/pmc_write.log 2>&1
python tools/pmc_traffic.py gpurun_out/pmc_fetch/p_counter_collection.csv gpurun_out/pmc_write/p_counter_collection.csv gpurun_out/pmc_traffic_fwd.json 8 256
timeout -k 10 400 python bench.py --traffic-file gpurun_out/pmc_traffic_fwd.json > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err
