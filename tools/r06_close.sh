#!/bin/bash
# Round-6 closing run on the phase-split build (gpurun_out/${T}_*):
#   the -m gpu suite and smoke(); re-tune of the training cache's forward 5x5/s2 shapes and
#   config-3 A/B lines (committed vs re-tuned cache, alternated); the bench lines (config 2
#   default with the CPU baseline, config 1, 4, RGBA); rocprofv3 --kernel-trace --stats of the
#   default bench command; a config-2 forward graph trace.  Stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -e
mkdir -p gpurun_out
T=${T:-r06i}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1
tail -n 1 gpurun_out/${T}_gputest.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1
tail -n 2 gpurun_out/${T}_smoke.txt
python tools/tune_drop.py profiles/tune_train_bf16_b16_256.json gpurun_out/${T}_tin_c3.json \
    1/0/5/2/16x64x64/192/192/False/g1 1/1/5/2/16x32x32/192/192/False/g1
timeout -k 10 400 python -u bench.py --train --steps 10 --no-cpu-baseline --no-dp-train \
    --tune-cache gpurun_out/${T}_tin_c3.json --save-tune gpurun_out/${T}_tune_train_bf16_b16_256.json \
    > gpurun_out/${T}_tune_c3.json 2> gpurun_out/${T}_tune_c3.err
python - "$T" <<'PY'
import json, sys
T = sys.argv[1]
old = json.load(open("profiles/tune_train_bf16_b16_256.json"))
new = json.load(open(f"gpurun_out/{T}_tune_train_bf16_b16_256.json"))
print("c3 retune", {k: (old.get(k), v) for k, v in new.items() if old.get(k) != v})
PY
for i in 1 2; do
  for v in old new; do
    if [ $v = old ]; then C=profiles/tune_train_bf16_b16_256.json; else C=gpurun_out/${T}_tune_train_bf16_b16_256.json; fi
    timeout -k 10 300 python -u bench.py --train --no-cpu-baseline --no-dp-train --tune-cache $C > gpurun_out/${T}_c3_${v}_${i}.json 2>> gpurun_out/${T}_c3ab.err
    echo "c3 $v run $i: $(cut -c 90-150 gpurun_out/${T}_c3_${v}_${i}.json)"
  done
done
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_c2.json 2> gpurun_out/${T}_c2.err
echo "c2: $(cut -c 90-190 gpurun_out/${T}_c2.json)"
timeout -k 10 300 python -u bench.py --alpha > gpurun_out/${T}_c1.json 2> gpurun_out/${T}_c1.err
echo "c1: $(cut -c 90-190 gpurun_out/${T}_c1.json)"
timeout -k 10 400 python -u bench.py --size 1024 --batch 4 --no-dp-train > gpurun_out/${T}_c4.json 2> gpurun_out/${T}_c4.err
echo "c4: $(cut -c 90-190 gpurun_out/${T}_c4.json)"
timeout -k 10 300 python -u bench.py --rgba --no-cpu-baseline > gpurun_out/${T}_rgba.json 2> gpurun_out/${T}_rgba.err
echo "rgba: $(cut -c 90-190 gpurun_out/${T}_rgba.json)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_bench -o b -- python bench.py --no-cpu-baseline > gpurun_out/${T}_prof_bench.log 2>&1
echo "rocprof done"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_tr_c2 -o t -- python tools/graph_trace.py --reps 20 > gpurun_out/${T}_tr_c2.log 2>&1
python tools/graph_trace.py --analyze gpurun_out/${T}_tr_c2/t_kernel_trace.csv > gpurun_out/${T}_tr_c2.txt
head -n 1 gpurun_out/${T}_tr_c2.txt
