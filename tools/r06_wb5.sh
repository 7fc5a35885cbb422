#!/bin/bash
# round 6: window block stage probes + rocprofv3 kernel trace of the A/B probe, then the
# training tests.  Stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 python -u tools/winblock3_stage_probe.py --config 2 > gpurun_out/r06_wb5_stage_c2.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/winblock3_stage_probe.py --config 4 > gpurun_out/r06_wb5_stage_c4.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_wb5_prof -o wb5 -- \
  python3 tools/winblock3_probe.py --reps 2 --variants v3 > gpurun_out/r06_wb5_prof.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train.py > gpurun_out/r06_train_tests.log 2>&1 || exit $?
