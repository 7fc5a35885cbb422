# Round-3 final GPU session, part 2: configs 3 and 4, the RGBA pipeline, and rocprofv3 kernel
# stats of the default bench command (no CPU baseline).
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03v6}
timeout -k 10 400 python bench.py --train > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err
timeout -k 10 400 python bench.py --size 1024 --batch 4 --no-dp-train > gpurun_out/${TAG}_c4.json 2> gpurun_out/${TAG}_c4.err
timeout -k 10 300 python bench.py --rgba --no-cpu-baseline > gpurun_out/${TAG}_rgba.json 2> gpurun_out/${TAG}_rgba.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o b -- python bench.py --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
