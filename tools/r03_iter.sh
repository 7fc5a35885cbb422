# One build -> measure iteration: the conv-tile GPU tests touched by the change, then the
# retune + config-2 line with its kernel table (tools/r03_retune.sh).  Outputs gpurun_out/.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03i}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${TESTK:-pw_tile or wstream or patch_tiles}" > gpurun_out/${TAG}_tests.log 2>&1
TAG=${TAG} bash tools/r03_retune.sh
