#!/bin/bash
# PMC passes of the config-2 forward on the phase-split build (traffic per dispatch + MFMA busy,
# tools/pmc_fwd.sh), copied into profiles/ on the box so the bench line's roofline reads them;
# then the default bench line, and rocprofv3 --kernel-trace --stats of a forward-only bench
# command (the dominant kernel's average without the training launches of the same name).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -e
mkdir -p gpurun_out
T=${T:-r06j}
TAG=${T} bash tools/pmc_fwd.sh
cp gpurun_out/${T}_pmc_traffic_fwd.json profiles/r06_pmc_traffic_fwd.json
cp gpurun_out/${T}_pmc_mfma_fwd.txt profiles/r06_pmc_mfma_fwd.txt
echo "pmc done"
grep -E "conv_patch|splitk|mse_partial|conv_fpatch_kernel<4, 128, 4, 4, 7" gpurun_out/${T}_pmc_mfma_fwd.txt | head -n 12
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_c2.json 2> gpurun_out/${T}_c2.err
echo "c2: $(cut -c 90-190 gpurun_out/${T}_c2.json)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_fwd -o b -- python bench.py --no-cpu-baseline --no-dp-train --no-parity-mode > gpurun_out/${T}_prof_fwd.log 2>&1
grep -E "conv_patch_kernel<8, 192, 2, 4, 4, false>" gpurun_out/${T}_prof_fwd/b_kernel_stats.csv | cut -c 1-160
