#!/bin/bash
# round 6: window block tests, graph-replay A/B against the round-3 kernel, stage probes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py -k "winblock_head_pair or winattn_block" > gpurun_out/r06_wb6_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/winblock3_probe.py > gpurun_out/r06_wb6_probe.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/winblock3_stage_probe.py --config 2 > gpurun_out/r06_wb6_stage_c2.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/winblock3_stage_probe.py --config 4 > gpurun_out/r06_wb6_stage_c4.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_wb6_prof -o wb6 -- \
  python3 tools/winblock3_probe.py --reps 2 --variants v3 > gpurun_out/r06_wb6_prof.log 2>&1 || exit $?
