# Round-5 check (GPU box): the batch-split forward (tests), then interleaved forward A/Bs of
# RGBAC_BATCH_SPLIT 1 vs 2 and 1 vs 4.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_models.py -x -q -s -k "split or bf16" --timeout 240 --timeout-method thread > gpurun_out/r05j_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^split|passed|failed|Error" gpurun_out/r05j_tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
VAR=RGBAC_BATCH_SPLIT A=1 B=2 TAG=split bash tools/ab_env.sh; rc=$?; [ $rc -eq 0 ] || exit $rc
VAR=RGBAC_BATCH_SPLIT A=1 B=4 TAG=split4 bash tools/ab_env.sh
