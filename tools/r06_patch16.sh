#!/bin/bash
# 16-row patch tiles and the phase split of the 5x5/s2 convs (gpurun_out/${T}_*):
#   1. patch-tile tests + the glue-kernel tests around them;
#   2. tools/patch_probe.py on the four strided shapes (parity vs the first candidate, times);
#   3. re-tune the /5/2/ launch shapes of the config-2 / config-4 tile caches inside the bench
#      (L2-flushed candidate timing), then forward-only A/B lines: old cache vs re-tuned cache;
#   4. a config-2 forward graph trace on the re-tuned cache.
# Stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -e
mkdir -p gpurun_out
T=${T:-r06p}
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_ops.py -k "patch_tiles or finalize or splitk or split_k" -m gpu > gpurun_out/${T}_tests.txt 2>&1
tail -n 2 gpurun_out/${T}_tests.txt
timeout -k 10 200 python -u tools/patch_probe.py --shape s2 > gpurun_out/${T}_probe.txt 2>&1
timeout -k 10 200 python -u tools/patch_probe.py --shape convT >> gpurun_out/${T}_probe.txt 2>&1
cat gpurun_out/${T}_probe.txt
python tools/tune_drop.py profiles/tune_fwd_bf16_b8_256.json gpurun_out/${T}_tin_c2.json /5/2/
python tools/tune_drop.py profiles/tune_fwd_bf16_b4_1024.json gpurun_out/${T}_tin_c4.json /5/2/
timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --no-dp-train --no-parity-mode \
    --tune-cache gpurun_out/${T}_tin_c2.json --save-tune gpurun_out/${T}_tune_fwd_bf16_b8_256.json \
    > gpurun_out/${T}_tune_c2.json 2> gpurun_out/${T}_tune_c2.err
timeout -k 10 300 python -u bench.py --size 1024 --batch 4 --steps 10 --no-cpu-baseline --no-dp-train \
    --no-parity-mode --tune-cache gpurun_out/${T}_tin_c4.json --save-tune gpurun_out/${T}_tune_fwd_bf16_b4_1024.json \
    > gpurun_out/${T}_tune_c4.json 2> gpurun_out/${T}_tune_c4.err
python - "$T" <<'PY'
import json, sys
T = sys.argv[1]
for c, f in (("c2", "tune_fwd_bf16_b8_256"), ("c4", "tune_fwd_bf16_b4_1024")):
    old = json.load(open(f"profiles/{f}.json")); new = json.load(open(f"gpurun_out/{T}_{f}.json"))
    print(c, {k: (old.get(k), v) for k, v in new.items() if "/5/2/" in k})
PY
for i in 1 2; do
  for v in old new; do
    if [ $v = old ]; then C=profiles/tune_fwd_bf16_b8_256.json; else C=gpurun_out/${T}_tune_fwd_bf16_b8_256.json; fi
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-parity-mode --no-dp-train --steps 50 --tune-cache $C > gpurun_out/${T}_ab_${v}_${i}.json 2>> gpurun_out/${T}_ab.err
    echo "c2 $v run $i: $(cut -c 60-140 gpurun_out/${T}_ab_${v}_${i}.json)"
  done
done
for v in old new; do
  if [ $v = old ]; then C=profiles/tune_fwd_bf16_b4_1024.json; else C=gpurun_out/${T}_tune_fwd_bf16_b4_1024.json; fi
  timeout -k 10 200 python -u bench.py --size 1024 --batch 4 --no-cpu-baseline --no-parity-mode --no-dp-train --steps 10 --tune-cache $C > gpurun_out/${T}_ab4_${v}.json 2>> gpurun_out/${T}_ab.err
  echo "c4 $v: $(cut -c 60-140 gpurun_out/${T}_ab4_${v}.json)"
done
