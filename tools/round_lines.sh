# Round-end bench lines (GPU only; outputs under gpurun_out/): config 2 (default, with the CPU
# baseline and fp32 parity line), config 3 (--train), config 4 (--size 1024 --batch 4), the
# RGBA pipeline (--rgba), and rocprofv3 kernel-trace stats of the default command.
export TMPDIR=/tmp
set -e
timeout -k 10 300 python bench.py > gpurun_out/line_c2.json 2> gpurun_out/line_c2.err
timeout -k 10 400 python bench.py --train > gpurun_out/line_c3.json 2> gpurun_out/line_c3.err
timeout -k 10 400 python bench.py --size 1024 --batch 4 > gpurun_out/line_c4.json 2> gpurun_out/line_c4.err
timeout -k 10 300 python bench.py --rgba --no-cpu-baseline > gpurun_out/line_rgba.json 2> gpurun_out/line_rgba.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o b -- python bench.py --no-cpu-baseline > gpurun_out/prof_c2.log 2>&1
