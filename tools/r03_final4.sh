# Round-3 closing GPU session: the whole -m gpu suite, smoke(), the config-2 default line and
# the config-3 line (CPU baselines included), training rocprofv3 kernel stats.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03v9}
timeout -k 10 560 python -u -m pytest tests -m gpu -v -x --timeout 100 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err
timeout -k 10 240 python bench.py --train > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_tprof -o t -- python bench.py --train --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_tprof.log 2>&1
