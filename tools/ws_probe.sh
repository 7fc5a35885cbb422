export TMPDIR=/tmp
for T in 35,1 6,1 26,1 33,4; do
  echo "== lrp3 128->8 tile $T"
  timeout -k 10 60 python tools/conv_probe.py --cin 128 --cout 8 --k 3 --hw 32 --act none --only $T --iters 30 2>&1 | grep -v amdgpu.ids
  echo "== 256->16 tile $T"
  timeout -k 10 60 python tools/conv_probe.py --cin 256 --cout 16 --k 3 --hw 32 --act none --only $T --iters 30 2>&1 | grep -v amdgpu.ids
done
