#!/bin/bash
# Re-check of a rebuilt tree on one box (outputs under gpurun_out/r06r_*): the -m gpu suite,
# smoke(), the default bench line, then A/B pairs of the fused prologue / finalize and of the
# in-launch split-K (two short forward-only lines each way, alternated).  Stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -e
mkdir -p gpurun_out
T=${T:-r06r}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1
tail -n 3 gpurun_out/${T}_gputest.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1
tail -n 2 gpurun_out/${T}_smoke.txt
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_c2.json 2> gpurun_out/${T}_c2.err
cut -c 1-300 gpurun_out/${T}_c2.json
# A/B pairs, alternated: $1 = env knob, values 0 / 1
ab() {
  for i in 1 2; do
    for v in 0 1; do
      env $1=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-parity-mode --no-dp-train --steps 50 > gpurun_out/${T}_$1_${v}_${i}.json 2>> gpurun_out/${T}_ab.err
      echo "$1=$v run $i: $(cut -c 1-160 gpurun_out/${T}_$1_${v}_${i}.json)"
    done
  done
}
ab RGBAC_FUSED_PROLOGUE
ab RGBAC_INLAUNCH_SPLITK
