# winblock iteration: fused-block tests, then probe timings at the config-2 and config-4 sizes.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03wb}
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread -k "winattn or winblock or win_" > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 120 python tools/winblock_probe.py > gpurun_out/${TAG}_probe.log 2>&1
timeout -k 10 120 python tools/winblock_probe.py --alpha ones >> gpurun_out/${TAG}_probe.log 2>&1
timeout -k 10 120 python tools/winblock_probe.py --alpha ones --batch 4 --size 256 >> gpurun_out/${TAG}_probe.log 2>&1
timeout -k 10 120 python tools/winblock_probe.py --batch 4 --size 256 >> gpurun_out/${TAG}_probe.log 2>&1
