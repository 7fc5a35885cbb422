# A/B: slice-chain side-stream precompute of the wide tail wave (RGBAC_SLICE_PRECOMPUTE=tail)
# against the default, interleaved, config 2 (no CPU baseline / parity / dp_train).
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03ab}
timeout -k 10 200 python -u -m pytest tests/test_gpu_models.py -m gpu -x -q --timeout 100 --timeout-method thread -k "precompute" > gpurun_out/${TAG}_test.log 2>&1
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 100 --timeout-method thread -k "pw_tile or smallk or gdn" > gpurun_out/${TAG}_pwtest.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-dp-train --no-cpu-baseline --no-parity-mode > gpurun_out/${TAG}_base$i.json 2>> gpurun_out/${TAG}.err
  RGBAC_SLICE_PRECOMPUTE=tail timeout -k 10 200 python bench.py --no-dp-train --no-cpu-baseline --no-parity-mode > gpurun_out/${TAG}_tail$i.json 2>> gpurun_out/${TAG}.err
done
RGBAC_SLICE_PRECOMPUTE=tail timeout -k 10 200 python bench.py --no-dp-train --no-cpu-baseline --no-parity-mode --layers gpurun_out/${TAG}_tail_layers.txt > gpurun_out/${TAG}_tail3.json 2>> gpurun_out/${TAG}.err
