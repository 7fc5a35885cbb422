# One-launch concatenation copies: train tests, then config 3 with and without (same box).
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q --timeout 100 --timeout-method thread > gpurun_out/cat_test.log 2>&1
timeout -k 10 200 python bench.py --train --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/cat_c3_multi.json 2> gpurun_out/cat_c3_multi.err
RGBAC_CAT_MULTI=0 timeout -k 10 200 python bench.py --train --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/cat_c3_single.json 2> gpurun_out/cat_c3_single.err
timeout -k 10 200 python bench.py --train --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/cat_c3_multi2.json 2> gpurun_out/cat_c3_multi2.err
RGBAC_CAT_MULTI=0 timeout -k 10 200 python bench.py --train --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/cat_c3_single2.json 2> gpurun_out/cat_c3_single2.err
