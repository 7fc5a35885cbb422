# Round-5 check (GPU box): loss-pass changes (finalize blocks / chains) -- the ops, model,
# north-star and training tests, then a config-4 forward trace.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_northstar.py tests/test_gpu_train.py tests/test_gpu_rgba.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r05i_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r05i_tests.log; [ $rc -eq 0 ] || exit $rc
d=gpurun_out/r05i_c4
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o t -- python tools/graph_trace.py --batch 4 --size 1024 --reps 6 > $d.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
python tools/graph_trace.py --analyze $d/t_kernel_trace.csv > $d.txt; head -1 $d.txt; grep -E "mse|finalize" $d.txt | head -4
