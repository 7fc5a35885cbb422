# Round-5 fold check (GPU box): fold kernel tests, then ops/train, the bf16 model tests and an
# interleaved A/B of the forward graph with RGBAC_FOLD on / off.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_ops.py -k "fold or bits" -x -q --timeout 120 --timeout-method thread > gpurun_out/r05e_fold.log 2>&1
rc=$?; echo "fold rc=$rc"; tail -5 gpurun_out/r05e_fold.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_models.py -x -q -s -k "bf16" --timeout 200 --timeout-method thread > gpurun_out/r05e_models.log 2>&1
rc=$?; echo "models rc=$rc"; grep -E "^fold|passed|failed" gpurun_out/r05e_models.log | tail -3; [ $rc -eq 0 ] || exit $rc
VAR=RGBAC_FOLD A=1 B=0 TAG=fold2 bash tools/ab_env.sh; rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
VAR=RGBAC_FOLD_BN1 A=64 B=128 TAG=foldbn bash tools/ab_env.sh; rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_northstar.py tests/test_gpu_parity.py tests/test_gpu_codec.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05e_tests.log 2>&1
rc=$?; echo "model-suite rc=$rc"; tail -3 gpurun_out/r05e_tests.log; exit $rc
