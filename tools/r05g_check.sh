# Round-5 check (GPU box): the patch-kernel tests and the model tests with the spatial-major
# XCD placement (RGBAC_XCD_REMAP=2), then interleaved forward A/Bs: the placement (1 vs 2) and
# the in-graph-tuned tile cache.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
RGBAC_XCD_REMAP=2 timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_parity.py tests/test_gpu_fold.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05g_tests.log 2>&1
rc=$?; echo "tests(remap 2) rc=$rc"; tail -2 gpurun_out/r05g_tests.log; [ $rc -eq 0 ] || exit $rc
VAR=RGBAC_XCD_REMAP A=1 B=2 TAG=xcd bash tools/ab_env.sh; rc=$?; [ $rc -eq 0 ] || exit $rc
VAR=RGBAC_TUNE_CACHE A=profiles/tune_fwd_bf16_b8_256.json B=tools/tune_alt_c2.json TAG=gt bash tools/ab_env.sh
