# r3hp: heavy_pixel_factor 30 / 40 / 50 / 65 at N = 1, D = 4 on the final build,
# interleaved twice at 200 steps and once at 20.
set -u
O=gpurun_out/r3hp
mkdir -p $O
for rep in a b; do
  for f in 30 40 50 65; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie --steps 200 --set heavy_pixel_factor=$f > $O/f${f}_$rep.json 2> $O/f${f}_$rep.err || exit $?
  done
done
for f in 30 40 50 65; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie --steps 20 --set heavy_pixel_factor=$f > $O/f${f}_20.json 2> $O/f${f}_20.err || exit $?
done
echo done > $O/done.txt
