# Round bench lines (GPU only; outputs under gpurun_out/<TAG>_*): smoke, config 2 (default: CPU
# baseline, fp32 parity line with symbol accounting, dp_train sub-record), config 1 (--alpha),
# config 3 (--train), config 4 (--size 1024 --batch 4), the RGBA pipeline (--rgba).
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03}
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err
timeout -k 10 300 python bench.py --alpha > gpurun_out/${TAG}_c1.json 2> gpurun_out/${TAG}_c1.err
timeout -k 10 400 python bench.py --train > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err
timeout -k 10 500 python bench.py --size 1024 --batch 4 --no-dp-train > gpurun_out/${TAG}_c4.json 2> gpurun_out/${TAG}_c4.err
timeout -k 10 300 python bench.py --rgba --no-cpu-baseline > gpurun_out/${TAG}_rgba.json 2> gpurun_out/${TAG}_rgba.err
