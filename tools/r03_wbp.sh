# Fused attention blocks: tests and probe timings (config-2 and config-4 attention sizes).
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03wp}
timeout -k 10 200 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -v --timeout 100 --timeout-method thread -k "winattn_block" -s > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 120 python tools/winblock_probe.py > gpurun_out/${TAG}_probe.log 2>&1
timeout -k 10 120 python tools/winblock_probe.py --alpha ones --batch 4 --size 256 >> gpurun_out/${TAG}_probe.log 2>&1
