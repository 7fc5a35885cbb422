# MFMA attention-core backward: train tests + attention-layer tests, then config 3 with the
# MFMA and the VALU backward (same box), each with a per-layer table.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_layers.py -m gpu -x -q --timeout 100 --timeout-method thread > gpurun_out/abwd_test.log 2>&1
timeout -k 10 300 python bench.py --train --steps 10 --warmup 3 --no-cpu-baseline --layers gpurun_out/abwd_layers_mfma.txt > gpurun_out/abwd_c3_mfma.json 2> gpurun_out/abwd_c3_mfma.err
RGBAC_ATTN_BWD_VALU=1 timeout -k 10 300 python bench.py --train --steps 10 --warmup 3 --no-cpu-baseline --layers gpurun_out/abwd_layers_valu.txt > gpurun_out/abwd_c3_valu.json 2> gpurun_out/abwd_c3_valu.err
timeout -k 10 300 python bench.py --train --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abwd_c3_mfma2.json 2> gpurun_out/abwd_c3_mfma2.err
