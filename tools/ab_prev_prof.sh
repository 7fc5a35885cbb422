#!/bin/bash
# per-kernel forward times of two library builds on one box (rocprofv3 kernel trace of the
# default bench run): the working tree's library and rgbac/librgbac_hip_prev.so
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
P=$GRAFT_REPO_ROOT/deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd/rgbac/librgbac_hip_prev.so
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_fwd_new -o fwd -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --no-cpu-baseline --no-dp-train > $GRAFT_REPO_ROOT/gpurun_out/prof_fwd_new.log 2>&1
RGBAC_LIB_PATH=$P timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_fwd_old -o fwd -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --no-cpu-baseline --no-dp-train > $GRAFT_REPO_ROOT/gpurun_out/prof_fwd_old.log 2>&1
cd $GRAFT_REPO_ROOT
for v in new old; do
  python3 tools/prof_db_stats.py gpurun_out/prof_fwd_$v/fwd_results.db --steps 25 --top 60 --csv gpurun_out/prof_fwd_$v.csv > gpurun_out/prof_fwd_$v.txt
  rm -rf gpurun_out/prof_fwd_$v
done
