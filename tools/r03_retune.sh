# Re-tune the committed forward tile caches (config 2, config 4) with the current tile set,
# then the config-2 line with the per-layer kernel table.  Outputs under gpurun_out/.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03t}
timeout -k 10 400 python bench.py --tune-cache '' --save-tune profiles/tune_fwd_bf16_b8_256.json --no-cpu-baseline --no-dp-train --no-parity-mode > gpurun_out/${TAG}_tune_c2.json 2> gpurun_out/${TAG}_tune_c2.err
timeout -k 10 500 python bench.py --size 1024 --batch 4 --tune-cache '' --save-tune profiles/tune_fwd_bf16_b4_1024.json --no-cpu-baseline --no-dp-train --no-parity-mode > gpurun_out/${TAG}_tune_c4.json 2> gpurun_out/${TAG}_tune_c4.err
cp profiles/tune_fwd_bf16_b8_256.json profiles/tune_fwd_bf16_b4_1024.json gpurun_out/
timeout -k 10 400 python bench.py --kernels --layers gpurun_out/${TAG}_layers.txt --no-cpu-baseline --no-dp-train > gpurun_out/${TAG}_c2k.json 2> gpurun_out/${TAG}_c2k.err
