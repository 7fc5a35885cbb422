# Round profile of the default bench command: bench line, rocprofv3 kernel-trace stats of the
# SAME command, PMC HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes over the graph
# replay); GPU only.  Outputs under gpurun_out/.
export TMPDIR=/tmp
set -e
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o b -- python bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o p -- python tools/graph_trace.py --reps 5 > gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o p -- python tools/graph_trace.py --reps 5 > gpurun_out/pmc_write.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ktrace -o t -- python tools/graph_trace.py --reps 20 > gpurun_out/ktrace.log 2>&1
