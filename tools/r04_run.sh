set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k "winattn_block or stem or patch_tiles or attn" > gpurun_out/r04_t3.log 2>&1
timeout -k 10 120 python -u tools/winblock_stage_probe.py --batch 8 --size 64 > gpurun_out/r04_wb_probe_v2.txt 2>&1
timeout -k 10 200 python -u tools/data_probe.py --pipeline > gpurun_out/r04_data_pipeline.json 2> gpurun_out/r04_data_pipeline.err
timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --no-dp-train --layers gpurun_out/r04_layers_c2_v2.txt > gpurun_out/r04_c2_v2.json 2> gpurun_out/r04_c2_v2.err
TAG=r04_v2 bash tools/pmc_fwd.sh
