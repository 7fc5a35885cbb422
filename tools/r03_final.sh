# Round-3 final GPU session, part 1: the whole -m gpu suite (verbose), smoke(), config 2
# (default bench: CPU baseline, fp32 parity block, dp_train) and config 1.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03v6}
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 100 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err
timeout -k 10 300 python bench.py --alpha > gpurun_out/${TAG}_c1.json 2> gpurun_out/${TAG}_c1.err
