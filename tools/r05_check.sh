#!/bin/bash
# Round-5 check: the changed-kernel tests, a forward graph trace, the pointwise probe
# (RGBAC_PW2_ALL A/B), then (RETUNE=1) the slice-chain tile retune.  GPU only.
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_northstar.py tests/test_gpu_rgba.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gt_${TAG} -o t -- python tools/graph_trace.py --reps 20 > gpurun_out/gt_${TAG}.log 2>&1 || exit 3
python tools/graph_trace.py --analyze gpurun_out/gt_${TAG}/t_kernel_trace.csv > gpurun_out/${TAG}_graph_trace.txt
head -1 gpurun_out/${TAG}_graph_trace.txt
timeout -k 10 120 python tools/pw_probe.py > gpurun_out/${TAG}_pw_probe.txt 2>&1 || exit 4
RGBAC_PW2_ALL=1 timeout -k 10 120 python tools/pw_probe.py >> gpurun_out/${TAG}_pw_probe.txt 2>&1 || exit 4
grep PW2 gpurun_out/${TAG}_pw_probe.txt
if [ "${RETUNE:-0}" = "1" ]; then
  PATTERN=1/0/3/1/8x32x32 TAG=${TAG}_kschain timeout -k 10 900 bash tools/retune.sh > gpurun_out/${TAG}_retune.log 2>&1
  echo "retune rc=$?"
  tail -c 250 gpurun_out/${TAG}_kschain_c2.json
fi
