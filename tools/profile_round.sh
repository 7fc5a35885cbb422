# Round profile: default bench line (config 2, with CPU baseline), rocprofv3 kernel-trace stats
# of the SAME command, PMC HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes over the graph
# replay), per-dispatch graph trace, training bench (config 3) and 1024^2 bench (config 4).
# GPU only; outputs under gpurun_out/.
export TMPDIR=/tmp
set -e
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o b -- python bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o p -- python tools/graph_trace.py --reps 5 > gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o p -- python tools/graph_trace.py --reps 5 > gpurun_out/pmc_write.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ktrace -o t -- python tools/graph_trace.py --reps 20 > gpurun_out/ktrace.log 2>&1
if [ "${WITH_TRAIN:-1}" = "1" ]; then
  timeout -k 10 500 python bench.py --train --layers gpurun_out/layers_train.txt > gpurun_out/bench_train.json 2> gpurun_out/bench_train.err
  timeout -k 10 300 python bench.py --size 1024 --batch 4 --no-cpu-baseline > gpurun_out/bench_1024.json 2> gpurun_out/bench_1024.err
fi
