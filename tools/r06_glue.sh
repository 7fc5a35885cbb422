#!/bin/bash
# Latency-chain fixes in the forward's glue kernels (gpurun_out/${T}_*): the MSE pass and the
# split-K epilogue with their loads batched ahead of the (unchanged-order) adds.  Tests around
# them, one forward bench line (parity section: per-image bpp / PSNR against the last line's)
# and a config-2 forward graph trace.  Stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -e
mkdir -p gpurun_out
T=${T:-r06h}
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_northstar.py tests/test_gpu_parity.py -m gpu > gpurun_out/${T}_tests.txt 2>&1
tail -n 2 gpurun_out/${T}_tests.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-dp-train > gpurun_out/${T}_c2.json 2> gpurun_out/${T}_c2.err
echo "c2: $(cut -c 60-200 gpurun_out/${T}_c2.json)"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_tr_c2 -o t -- python tools/graph_trace.py --reps 20 > gpurun_out/${T}_tr_c2.log 2>&1
python tools/graph_trace.py --analyze gpurun_out/${T}_tr_c2/t_kernel_trace.csv > gpurun_out/${T}_tr_c2.txt
head -n 1 gpurun_out/${T}_tr_c2.txt
grep -E "mse_partial|splitk_epilogue|finalize" gpurun_out/${T}_tr_c2.txt | head -n 8
