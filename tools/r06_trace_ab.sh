#!/bin/bash
# Config-2 forward graph traces (rocprofv3 kernel trace, 20 replays) under candidate tile
# caches (tools/cand/*.json vs the committed one), then forward-only bench lines alternated.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -e
mkdir -p gpurun_out
T=${T:-r06t}
for v in base a b c; do
  if [ $v = base ]; then C=profiles/tune_fwd_bf16_b8_256.json; else C=tools/cand/c2_$v.json; fi
  RGBAC_TUNE_CACHE=$C timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_tr_$v -o t -- python tools/graph_trace.py --reps 20 > gpurun_out/${T}_tr_$v.log 2>&1
  python tools/graph_trace.py --analyze gpurun_out/${T}_tr_$v/t_kernel_trace.csv > gpurun_out/${T}_tr_$v.txt
  echo "$v: $(head -n 1 gpurun_out/${T}_tr_$v.txt)"
  grep -E "conv_patch|splitk_epilogue|mse_partial" gpurun_out/${T}_tr_$v.txt | head -n 12
done
for i in 1 2 3; do
  for v in base a; do
    if [ $v = base ]; then C=profiles/tune_fwd_bf16_b8_256.json; else C=tools/cand/c2_$v.json; fi
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-parity-mode --no-dp-train --steps 50 --tune-cache $C > gpurun_out/${T}_ab_${v}_${i}.json 2>> gpurun_out/${T}_ab.err
    echo "c2 $v run $i: $(cut -c 100-150 gpurun_out/${T}_ab_${v}_${i}.json)"
  done
done
