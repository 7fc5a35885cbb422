#!/bin/bash
# Round-6 closing run (GPU only; outputs under gpurun_out/r06f_*):
#   1. the full -m gpu suite and smoke();
#   2. PMC traffic passes for config 4 and config 3, copied into profiles/ on the box so the
#      bench lines below report them (and returned for committing);
#   3. every bench line (config 2 default with CPU baseline, config 1, 3, 4, RGBA);
#   4. rocprofv3 --kernel-trace --stats of the default bench command.
# Stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -e
mkdir -p gpurun_out
T=r06f
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1
bash tools/pmc_1024.sh
cp gpurun_out/pmc_traffic_fwd_b4_1024.json profiles/r06_pmc_traffic_fwd_b4_1024.json
bash tools/pmc_train.sh > gpurun_out/${T}_pmc_train.log 2>&1
cp gpurun_out/pmc_traffic_train.json profiles/r06_pmc_traffic_train.json
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_c2.json 2> gpurun_out/${T}_c2.err
timeout -k 10 300 python -u bench.py --alpha > gpurun_out/${T}_c1.json 2> gpurun_out/${T}_c1.err
timeout -k 10 400 python -u bench.py --train > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.err
timeout -k 10 500 python -u bench.py --size 1024 --batch 4 --no-dp-train > gpurun_out/${T}_c4.json 2> gpurun_out/${T}_c4.err
timeout -k 10 300 python -u bench.py --rgba --no-cpu-baseline > gpurun_out/${T}_rgba.json 2> gpurun_out/${T}_rgba.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_bench -o b -- python bench.py --no-cpu-baseline > gpurun_out/${T}_prof_bench.log 2>&1
