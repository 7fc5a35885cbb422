#!/bin/bash
# round 6: full -m gpu suite, smoke(), then the default bench line.  Stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-a}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_gputest_$TAG.txt 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke_$TAG.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r06_line_c2_$TAG.json 2> gpurun_out/r06_bench_$TAG.err || exit $?
if [ -n "$WITH_TRAIN" ]; then
  timeout -k 10 400 python -u bench.py --train > gpurun_out/r06_line_c3_$TAG.json 2> gpurun_out/r06_c3_$TAG.err || exit $?
fi
