#!/bin/bash
# Round-6 closing runs (GPU only; outputs under gpurun_out/r06f_*), in two gpurun calls:
#   PART=a  PMC passes: config-2 forward traffic + MFMA busy (tools/pmc_fwd.sh), config-4
#           traffic (tools/pmc_1024.sh), config-3 traffic (tools/pmc_train.sh), copied into
#           profiles/ on the box so the bench lines report them (and returned for committing);
#           then rocprofv3 --kernel-trace --stats of the default bench command;
#   PART=b  the full -m gpu suite, smoke(), and every bench line (config 2 default with the CPU
#           baseline, config 1, 3, 4, RGBA).
# Stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -e
mkdir -p gpurun_out
T=r06f
if [ "${PART:-a}" = "a" ]; then
  TAG=${T} bash tools/pmc_fwd.sh
  cp gpurun_out/${T}_pmc_traffic_fwd.json profiles/r06_pmc_traffic_fwd.json
  cp gpurun_out/${T}_pmc_mfma_fwd.txt profiles/r06_pmc_mfma_fwd.txt
  echo "pmc_fwd done"
  bash tools/pmc_1024.sh
  cp gpurun_out/pmc_traffic_fwd_b4_1024.json profiles/r06_pmc_traffic_fwd_b4_1024.json
  echo "pmc_1024 done"
  bash tools/pmc_train.sh > gpurun_out/${T}_pmc_train.log 2>&1
  cp gpurun_out/pmc_traffic_train.json profiles/r06_pmc_traffic_train.json
  echo "pmc_train done"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_bench -o b -- python bench.py --no-cpu-baseline > gpurun_out/${T}_prof_bench.log 2>&1
  echo "rocprof done"
else
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1
  tail -n 1 gpurun_out/${T}_gputest.txt
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1
  tail -n 2 gpurun_out/${T}_smoke.txt
  timeout -k 10 400 python -u bench.py > gpurun_out/${T}_c2.json 2> gpurun_out/${T}_c2.err
  echo "c2: $(cut -c 100-190 gpurun_out/${T}_c2.json)"
  timeout -k 10 300 python -u bench.py --alpha > gpurun_out/${T}_c1.json 2> gpurun_out/${T}_c1.err
  echo "c1: $(cut -c 100-190 gpurun_out/${T}_c1.json)"
  timeout -k 10 400 python -u bench.py --train > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.err
  echo "c3: $(cut -c 100-190 gpurun_out/${T}_c3.json)"
  timeout -k 10 400 python -u bench.py --size 1024 --batch 4 --no-dp-train > gpurun_out/${T}_c4.json 2> gpurun_out/${T}_c4.err
  echo "c4: $(cut -c 100-190 gpurun_out/${T}_c4.json)"
  timeout -k 10 300 python -u bench.py --rgba --no-cpu-baseline > gpurun_out/${T}_rgba.json 2> gpurun_out/${T}_rgba.err
  echo "rgba: $(cut -c 100-190 gpurun_out/${T}_rgba.json)"
fi
