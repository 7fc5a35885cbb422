# winblock phase-stamp probe (probe build librgbac_wbprof.so) at the config-4 and config-2 sizes
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03ws}
timeout -k 10 120 python tools/winblock_stage_probe.py > gpurun_out/${TAG}.log 2>&1
timeout -k 10 120 python tools/winblock_stage_probe.py --batch 8 --size 64 --alpha half >> gpurun_out/${TAG}.log 2>&1
