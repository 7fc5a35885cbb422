# Iteration: fused-block / DSE / model / RGBA tests, attention probe, config-2 line + layers.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03i3}
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_models.py tests/test_gpu_rgba.py tests/test_golden.py -m gpu -x -v --timeout 100 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 120 python tools/winblock_probe.py > gpurun_out/${TAG}_probe.log 2>&1
timeout -k 10 120 python tools/winblock_probe.py --alpha ones --batch 4 --size 256 >> gpurun_out/${TAG}_probe.log 2>&1
timeout -k 10 200 python bench.py --no-dp-train --no-cpu-baseline --no-parity-mode --layers gpurun_out/${TAG}_layers.txt > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err
timeout -k 10 200 python bench.py --no-dp-train --no-cpu-baseline --no-parity-mode > gpurun_out/${TAG}_c2b.json 2>> gpurun_out/${TAG}_c2.err
