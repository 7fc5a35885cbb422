# Iteration: RU stream kernel with W1 staged once per workgroup -- tests, per-kernel probe of
# both builds on one box, then interleaved config-2 A/B.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03i8}
BASE=deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd/rgbac/librgbac_base.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_layers.py tests/test_gpu_models.py -m gpu -x -q --timeout 100 --timeout-method thread -k "residual or stream or bf16 or noshift" > gpurun_out/${TAG}_tests.log 2>&1
for i in 1 2; do
  RGBAC_LIB_PATH=$BASE timeout -k 10 120 python tools/ru_probe.py --kind 0 >> gpurun_out/${TAG}_probeA.log 2>&1
  timeout -k 10 120 python tools/ru_probe.py --kind 0 >> gpurun_out/${TAG}_probeB.log 2>&1
done
TAG=${TAG}ab bash tools/ab_lib.sh
