#!/bin/bash
# Final check of the in-tree library at HEAD: the -m gpu suite, smoke(), the default bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -e
mkdir -p gpurun_out
T=${T:-r06l}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1
tail -n 1 gpurun_out/${T}_gputest.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1
tail -n 2 gpurun_out/${T}_smoke.txt
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_c2.json 2> gpurun_out/${T}_c2.err
echo "c2: $(cut -c 90-190 gpurun_out/${T}_c2.json)"
