# winblock iteration: fused-block tests, phase-stamp probe, timing probe, config-2 line.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03w2}
timeout -k 10 200 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -q --timeout 100 --timeout-method thread -k "winattn_block" > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 120 python tools/winblock_stage_probe.py > gpurun_out/${TAG}_stage.log 2>&1
timeout -k 10 120 python tools/winblock_probe.py > gpurun_out/${TAG}_probe.log 2>&1
timeout -k 10 120 python tools/winblock_probe.py --alpha ones --batch 4 --size 256 >> gpurun_out/${TAG}_probe.log 2>&1
timeout -k 10 200 python bench.py --no-dp-train --no-cpu-baseline --no-parity-mode > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err
