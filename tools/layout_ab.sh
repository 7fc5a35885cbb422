# A/B of conv_kernel stage layouts (alternative builds of librgbac_hip.so via RGBAC_LIB_PATH); GPU only.
# Usage: bash tools/layout_ab.sh lib1.so lib2.so ...   (paths relative to the package's rgbac/)
export TMPDIR=/tmp
PKG=deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd
export PYTHONPATH=$PWD/$PKG:$PWD
set -e
for L in "$@"; do
  export RGBAC_LIB_PATH=$PWD/$PKG/rgbac/$L
  echo "==== $L"
  for P in "--cin 224 --cout 128 --k 3 --hw 32 --groups 2" "--cin 192 --cout 192 --k 5 --stride 2 --hw 128 --act none" \
           "--cin 88 --cout 224 --k 3 --hw 32 --groups 2" "--cin 224 --cout 128 --k 3 --hw 32" \
           "--cin 256 --cout 288 --k 3 --hw 16 --groups 2" "--cin 192 --cout 576 --k 1 --hw 64 --act none"; do
    echo "== $P"
    timeout -k 10 120 python tools/conv_probe.py $P --iters 30 > gpurun_out/ab_${L}_$(echo $P | tr -d " -").txt
  done
  timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ab_$L.json 2>gpurun_out/ab_$L.err
  python -c "import json,sys;d=json.load(open('gpurun_out/ab_$L.json'));print('BENCH',d['value'],d['roofline']['avg_launch_us'])"
done
