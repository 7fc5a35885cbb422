#!/bin/bash
# Same-box A/B of one environment switch on the forward graph replay: rocprofv3 kernel traces
# of tools/graph_trace.py with VAR=A and VAR=B, interleaved twice; prints each replay span.
# Usage (GPU box): VAR=RGBAC_SIDE_STREAMS A=1 B=0 TAG=side bash tools/ab_env.sh
# (ARGS: extra graph_trace.py arguments, e.g. "--batch 4 --size 1024"; REPS: replays)
export TMPDIR=/tmp
mkdir -p gpurun_out
VAR=${VAR:?set VAR}; A=${A:?}; B=${B:?}; TAG=${TAG:-ab}
for rep in 1 2; do
  for v in $A $B; do
    lab=$(basename "$v" | tr '/.' '__')
    d=gpurun_out/ab_${TAG}_${lab}_${rep}
    ( export $VAR=$v; timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o t -- \
        python tools/graph_trace.py --reps ${REPS:-20} ${ARGS:-} > $d.log 2>&1 ) || exit 3
    python tools/graph_trace.py --analyze $d/t_kernel_trace.csv > ${d}.txt
    echo "$VAR=$v rep $rep: $(head -1 ${d}.txt)"
  done
done
