# Full -m gpu suite, verbose (a line per test), then smoke().
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03f}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 100 --timeout-method thread --durations=25 > gpurun_out/${TAG}_gputest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
