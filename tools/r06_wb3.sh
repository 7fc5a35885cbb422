#!/bin/bash
# round 6: head-pair window block -- graph-replay A/B against the round-3 kernel, then a
# rocprofv3 kernel trace of the same probe (per-kernel averages).  Stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u tools/winblock3_probe.py > gpurun_out/r06_wb3_probe.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_wb3_prof -o wb3 -- \
  python3 tools/winblock3_probe.py --reps 2 > gpurun_out/r06_wb3_prof.log 2>&1 || exit $?
