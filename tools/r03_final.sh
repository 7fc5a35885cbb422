# Round-3 final GPU session: the whole -m gpu suite (verbose), smoke(), the round lines
# (configs 1-4 + RGBA) and rocprofv3 kernel stats of the default bench command.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03v6}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 100 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1
TAG=$TAG bash tools/round_lines.sh
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o b -- python bench.py --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
