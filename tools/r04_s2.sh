#!/bin/bash
# round 4: full -m gpu suite, then re-tune the 5x5/s2 conv shapes (new polyphase patch tiles)
# for the forward (config 2 / 4) and training (config 3) caches, and time the three lines.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04_gputest_v2.txt 2>&1
python tools/tune_drop.py profiles/tune_fwd_bf16_b8_256.json gpurun_out/tin_c2.json 1/0/5/2/
python tools/tune_drop.py profiles/tune_fwd_bf16_b4_1024.json gpurun_out/tin_c4.json 1/0/5/2/
python tools/tune_drop.py profiles/tune_train_bf16_b16_256.json gpurun_out/tin_c3.json 1/0/5/2/
timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --tune-cache gpurun_out/tin_c2.json --save-tune gpurun_out/tune_fwd_bf16_b8_256.json --layers gpurun_out/r04_layers_c2_s2.txt > gpurun_out/r04_c2_s2.json 2> gpurun_out/r04_c2_s2.err
timeout -k 10 300 python -u bench.py --size 1024 --batch 4 --steps 10 --no-cpu-baseline --no-dp-train --no-parity-mode --tune-cache gpurun_out/tin_c4.json --save-tune gpurun_out/tune_fwd_bf16_b4_1024.json > gpurun_out/r04_c4_s2.json 2> gpurun_out/r04_c4_s2.err
timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline --tune-cache gpurun_out/tin_c3.json --save-tune gpurun_out/tune_train_bf16_b16_256.json > gpurun_out/r04_c3_s2.json 2> gpurun_out/r04_c3_s2.err
