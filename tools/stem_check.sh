set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ops.py -m gpu -k "stem" > gpurun_out/stem_tests.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/stem_c2 -o t -- python tools/graph_trace.py --reps 20 > gpurun_out/stem_c2.log 2>&1
python tools/graph_trace.py --analyze gpurun_out/stem_c2/t_kernel_trace.csv > gpurun_out/stem_c2.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/stem_c4 -o t -- python tools/graph_trace.py --reps 6 --batch 4 --size 1024 > gpurun_out/stem_c4.log 2>&1
python tools/graph_trace.py --analyze gpurun_out/stem_c4/t_kernel_trace.csv > gpurun_out/stem_c4.txt
