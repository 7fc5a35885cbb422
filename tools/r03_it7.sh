# Iteration: pw-kernel gate epilogue (batched residual quads) -- tests and tile probes.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03i7}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fused.py tests/test_gpu_models.py -m gpu -x -q --timeout 100 --timeout-method thread -k "pw or gate or gdn or smallk or noshift or bf16" > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 200 python tools/tile_probe.py --only gate > gpurun_out/${TAG}_probe.log 2>&1
timeout -k 10 200 python tools/tile_probe.py --only gdn >> gpurun_out/${TAG}_probe.log 2>&1
