#!/bin/bash
# Re-tune the training tile cache (config 3) from scratch on this box, then A/B the new cache
# against the committed one (interleaved).  Outputs: gpurun_out/tune_train_bf16_b16_256.json
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
python tools/tune_drop.py profiles/tune_train_bf16_b16_256.json gpurun_out/tin_c3.json "1/"
timeout -k 10 500 python -u bench.py --train --steps 10 --no-cpu-baseline --tune-cache gpurun_out/tin_c3.json \
    --save-tune gpurun_out/tune_train_bf16_b16_256.json > gpurun_out/rt3_tune.json 2> gpurun_out/rt3_tune.err
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline > gpurun_out/rt3_old$i.json 2> gpurun_out/rt3_old$i.err
  timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline --tune-cache gpurun_out/tune_train_bf16_b16_256.json \
      > gpurun_out/rt3_new$i.json 2> gpurun_out/rt3_new$i.err
done
