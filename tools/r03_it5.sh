# Iteration: stem tests + probe, config-2 lines.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03i5}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_golden.py -m gpu -x -q --timeout 100 --timeout-method thread -k "stem or bf16 or golden" > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 120 python tools/stem_probe.py > gpurun_out/${TAG}_stem.log 2>&1
timeout -k 10 200 python bench.py --no-dp-train --no-cpu-baseline --no-parity-mode > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err
timeout -k 10 200 python bench.py --no-dp-train --no-cpu-baseline --no-parity-mode > gpurun_out/${TAG}_c2b.json 2>> gpurun_out/${TAG}_c2.err
