#!/bin/bash
# Re-tune chosen launch shapes of the committed tile caches (after a new tile family became a
# candidate for them) and time the lines with the new choices.  GPU only; outputs under
# gpurun_out/ (tune_*.json to merge into profiles/, <TAG>_c2 / c4 / c3 bench lines).
# Usage: PATTERN=1/0/5/2/ TAG=r04_s2 bash tools/retune.sh
#   PATTERN: substring of the cache keys to drop (dtype/mode/ksize/stride/...: runtime.prepare)
set -e
mkdir -p gpurun_out
TAG=${TAG:-retune}
PATTERN=${PATTERN:?set PATTERN}
python tools/tune_drop.py profiles/tune_fwd_bf16_b8_256.json gpurun_out/tin_c2.json $PATTERN
python tools/tune_drop.py profiles/tune_fwd_bf16_b4_1024.json gpurun_out/tin_c4.json $PATTERN
python tools/tune_drop.py profiles/tune_train_bf16_b16_256.json gpurun_out/tin_c3.json $PATTERN
timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --tune-cache gpurun_out/tin_c2.json \
    --save-tune gpurun_out/tune_fwd_bf16_b8_256.json --layers gpurun_out/${TAG}_layers_c2.txt \
    > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err
timeout -k 10 300 python -u bench.py --size 1024 --batch 4 --steps 10 --no-cpu-baseline --no-dp-train \
    --no-parity-mode --tune-cache gpurun_out/tin_c4.json --save-tune gpurun_out/tune_fwd_bf16_b4_1024.json \
    > gpurun_out/${TAG}_c4.json 2> gpurun_out/${TAG}_c4.err
timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline --tune-cache gpurun_out/tin_c3.json \
    --save-tune gpurun_out/tune_train_bf16_b16_256.json > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err
