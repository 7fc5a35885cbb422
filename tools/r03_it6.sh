# Iteration: narrow patch tile for the decoder's subpel conv -- tests, retune of the x4 shape
# into the committed caches, then a same-box A/B against the previous build.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03i6}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_golden.py tests/test_gpu_fused.py tests/test_gpu_rgba.py -m gpu -x -q --timeout 100 --timeout-method thread -k "patch or subpel or bf16 or golden or dse or rgba or wstream" > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 300 python bench.py --no-dp-train --no-cpu-baseline --no-parity-mode --save-tune gpurun_out/${TAG}_tune_b8_256.json --layers gpurun_out/${TAG}_layers.txt > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err
timeout -k 10 400 python bench.py --no-dp-train --no-cpu-baseline --no-parity-mode --size 1024 --batch 4 --save-tune gpurun_out/${TAG}_tune_b4_1024.json > gpurun_out/${TAG}_c4.json 2> gpurun_out/${TAG}_c4.err
