# Same-box sweep of runtime switches against the default, interleaved (config-2 lines).
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-sw}
run() { env $2 timeout -k 10 200 python bench.py --no-dp-train --no-cpu-baseline --no-parity-mode > gpurun_out/${TAG}_$1.json 2>> gpurun_out/${TAG}.err; }
run base1 ""
run splitk "RGBAC_INLAUNCH_SPLITK=1"
run base2 ""
run nw1 "RGBAC_WINBLOCK4_NW=1"
run base3 ""
run nw4 "RGBAC_WINBLOCK4_NW=4"
run base4 ""
run stag2 "RGBAC_RU_STAGGER=2"
run base5 ""
