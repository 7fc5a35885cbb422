# One stacked gradient sum per multiply-used latent tensor: train tests, config 3 with and without.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q --timeout 100 --timeout-method thread > gpurun_out/fan_test.log 2>&1
timeout -k 10 200 python bench.py --train --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/fan_c3_on.json 2> gpurun_out/fan_c3_on.err
RGBAC_FAN_OUT=0 timeout -k 10 200 python bench.py --train --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/fan_c3_off.json 2> gpurun_out/fan_c3_off.err
timeout -k 10 200 python bench.py --train --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/fan_c3_on2.json 2> gpurun_out/fan_c3_on2.err
RGBAC_FAN_OUT=0 timeout -k 10 200 python bench.py --train --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/fan_c3_off2.json 2> gpurun_out/fan_c3_off2.err
