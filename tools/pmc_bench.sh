# HBM traffic (PMC) + kernel-trace stats of the forward graph replay; GPU only.
# Writes gpurun_out/pmc_fetch, gpurun_out/pmc_write, gpurun_out/ktrace.
export TMPDIR=/tmp
set -e
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o p -- python tools/graph_trace.py --reps 5 > gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o p -- python tools/graph_trace.py --reps 5 > gpurun_out/pmc_write.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ktrace -o t -- python tools/graph_trace.py --reps 20 > gpurun_out/ktrace.log 2>&1
