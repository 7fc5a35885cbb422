# Fast GELU derivative in act_bwd (bf16): train tests, then config 3 with and without (same box).
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q --timeout 100 --timeout-method thread > gpurun_out/gelu_test.log 2>&1
timeout -k 10 200 python bench.py --train --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/gelu_c3_fast.json 2> gpurun_out/gelu_c3_fast.err
RGBAC_GELU_BWD_EXACT=1 timeout -k 10 200 python bench.py --train --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/gelu_c3_exact.json 2> gpurun_out/gelu_c3_exact.err
timeout -k 10 200 python bench.py --train --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/gelu_c3_fast2.json 2> gpurun_out/gelu_c3_fast2.err
RGBAC_GELU_BWD_EXACT=1 timeout -k 10 200 python bench.py --train --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/gelu_c3_exact2.json 2> gpurun_out/gelu_c3_exact2.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gelu_tprof -o t -- python bench.py --train --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/gelu_tprof.log 2>&1
