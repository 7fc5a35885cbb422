# Iteration: touched conv-tile tests, 1x1 tile probe, RU GELU-vs-ReLU probe, retune + line.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03j}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${TESTK:-pw_tile or smallk or wstream or patch_tiles}" > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 300 python tools/tile_probe.py --only "${PROBE:-gdn}" > gpurun_out/${TAG}_probe.log 2>&1
timeout -k 10 200 python tools/tile_probe.py --only gate >> gpurun_out/${TAG}_probe.log 2>&1
timeout -k 10 200 python tools/tile_probe.py --only 16x16 >> gpurun_out/${TAG}_probe.log 2>&1
timeout -k 10 120 python tools/ru_probe.py --kind 0 > gpurun_out/${TAG}_ru.log 2>&1
timeout -k 10 120 python tools/ru_probe.py --kind 1 >> gpurun_out/${TAG}_ru.log 2>&1
TAG=${TAG} bash tools/r03_retune.sh
