# Timing of conv variants on the forward's hot shapes (all tiles); GPU only.
export TMPDIR=/tmp
set -e
for P in "--cin 224 --cout 128 --k 3 --hw 32 --groups 2" "--cin 256 --cout 16 --k 3 --hw 32 --act none" \
         "--cin 120 --cout 224 --k 3 --hw 32 --groups 10" "--cin 192 --cout 192 --k 5 --stride 2 --hw 128 --act none" \
         "--cin 128 --cout 8 --k 3 --hw 32 --act none"; do
  echo "== $P"
  timeout -k 10 120 python tools/conv_probe.py $P --iters 30
done
