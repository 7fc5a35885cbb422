#!/bin/bash
# One GPU session: the given pytest targets, then (unless a step crashed / hung) a bench run.
# Exit codes 0/1 of pytest (pass / test failures) continue; anything else (fault, abort,
# timeout) stops the session there.
set -u
mkdir -p gpurun_out
TESTS=${TESTS:-"tests -m gpu"}
BENCH_ARGS=${BENCH_ARGS:-""}
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -v --timeout 300 --timeout-method thread \
    > gpurun_out/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -n 40 gpurun_out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
if [ -n "$BENCH_ARGS" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
  brc=$?
  echo "bench rc=$brc"; tail -n 5 gpurun_out/bench.log
  exit $brc
fi
exit $rc
