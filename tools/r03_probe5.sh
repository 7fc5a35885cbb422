# Tile probe of the slice chain's wide-wave convs (g10 / g5) and the chain's g2 / g1 convs.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03p5}
timeout -k 10 300 python tools/tile_probe.py --only g10 > gpurun_out/${TAG}_probe.log 2>&1
timeout -k 10 300 python tools/tile_probe.py --only g5 >> gpurun_out/${TAG}_probe.log 2>&1
timeout -k 10 300 python tools/tile_probe.py --only "g2" >> gpurun_out/${TAG}_probe.log 2>&1
