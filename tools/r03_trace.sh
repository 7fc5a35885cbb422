# In-graph per-dispatch durations of the config-2 forward (rocprofv3 kernel trace of 20 graph
# replays delimited by spin kernels) + the analysis table.  Outputs under gpurun_out/.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03g}
rm -rf gpurun_out/${TAG}_kt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_kt -o t -- python tools/graph_trace.py --reps 20 > gpurun_out/${TAG}_kt.log 2>&1
python tools/graph_trace.py --analyze $(find gpurun_out/${TAG}_kt -name "*kernel_trace.csv") > gpurun_out/${TAG}_graph_trace.txt
