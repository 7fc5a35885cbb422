# Round-5 glue-kernel check (GPU box): layout conversions, finalize_ex, pyramid, the bf16/fp32
# model tests, then a kernel trace of the forward graph.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_northstar.py -x -q --timeout 200 --timeout-method thread -k "layout or finalize or pyramid or forward or fold or north" > gpurun_out/r05f_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05f_tests.log; [ $rc -eq 0 ] || exit $rc
d=gpurun_out/r05f_trace
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o t -- python tools/graph_trace.py --reps 20 > $d.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
python tools/graph_trace.py --analyze $d/t_kernel_trace.csv > $d.txt; head -3 $d.txt; grep -E "pyramid|nhwc|nchw|mse|finalize" $d.txt | head -8
