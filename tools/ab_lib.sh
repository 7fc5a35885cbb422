# Same-box A/B of two builds of the library: the default librgbac_hip.so (B) against
# RGBAC_LIB_PATH=$BASE (A), config-2 bench lines interleaved (differences of ~1 % are below
# the box-to-box spread, so only same-box pairs are compared).  Optional TESTK: a -k filter
# of GPU tests run on B first.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-ab}
BASE=${BASE:-deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd/rgbac/librgbac_base.so}
if [ -n "$TESTK" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 100 --timeout-method thread -k "$TESTK" > gpurun_out/${TAG}_tests.log 2>&1
fi
for i in 1 2 3; do
  env $A_ENV RGBAC_LIB_PATH=$BASE timeout -k 10 200 python bench.py --no-dp-train --no-cpu-baseline --no-parity-mode > gpurun_out/${TAG}_A$i.json 2>> gpurun_out/${TAG}.err
  timeout -k 10 200 python bench.py --no-dp-train --no-cpu-baseline --no-parity-mode > gpurun_out/${TAG}_B$i.json 2>> gpurun_out/${TAG}.err
done
