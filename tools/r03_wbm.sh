# Fused attention blocks: tests, probe timings (config-2 / config-4 attention sizes), then the
# default bench line with a per-layer table.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03wm}
timeout -k 10 200 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -v --timeout 100 --timeout-method thread -k "winattn_block" -s > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 120 python tools/winblock_probe.py > gpurun_out/${TAG}_probe.log 2>&1
timeout -k 10 120 python tools/winblock_probe.py --alpha ones >> gpurun_out/${TAG}_probe.log 2>&1
timeout -k 10 120 python tools/winblock_probe.py --alpha ones --batch 4 --size 256 >> gpurun_out/${TAG}_probe.log 2>&1
timeout -k 10 120 python tools/winblock_probe.py --batch 4 --size 256 >> gpurun_out/${TAG}_probe.log 2>&1
timeout -k 10 400 python bench.py --no-dp-train --no-cpu-baseline --no-parity-mode --layers gpurun_out/${TAG}_layers.txt > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err
