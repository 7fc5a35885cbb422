# small-K tile (34) vs the streaming tiles on the forward's HBM-bound shapes; GPU only.
export TMPDIR=/tmp

for P in "--cin 192 --cout 192 --k 1 --hw 128 --act gelu --res" "--cin 192 --cout 576 --k 1 --hw 64 --act none" \
         "--cin 3 --cout 192 --k 5 --stride 2 --hw 256 --act none" "--cin 3 --cout 32 --k 1 --hw 256 --act none" \
         "--cin 32 --cout 3 --k 1 --hw 256 --act none --res"; do
  for T in 34,1 2,1; do
    case "$P" in *"--k 5"*) [ "$T" = "34,1" ] && continue;; esac
    echo "== $P tile $T"
    timeout -k 10 60 python tools/conv_probe.py $P --batch 8 --only $T --iters 30 2>&1 | grep -v amdgpu.ids
  done
done
