#!/bin/bash
# Forward graph traces of config 2 and config 4 (rocprofv3 kernel trace, per-kernel table).
# GPU only; gpurun_out/${TAG}_c2.txt, ${TAG}_c4.txt.  TESTS: optional pytest -k filter run first.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-tr}
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu -k "$TESTS" > gpurun_out/${TAG}_tests.log 2>&1
fi
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_c2 -o t -- python tools/graph_trace.py --reps 20 > gpurun_out/${TAG}_c2.log 2>&1
python tools/graph_trace.py --analyze gpurun_out/${TAG}_c2/t_kernel_trace.csv > gpurun_out/${TAG}_c2.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_c4 -o t -- python tools/graph_trace.py --reps 6 --batch 4 --size 1024 > gpurun_out/${TAG}_c4.log 2>&1
python tools/graph_trace.py --analyze gpurun_out/${TAG}_c4/t_kernel_trace.csv > gpurun_out/${TAG}_c4.txt
