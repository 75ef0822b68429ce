# r3n: option order_split (only the costliest tiles first, the rest in raster
# order) against the full cost order, one frame per launch and 8 per launch.
set -u
O=gpurun_out/r3n
mkdir -p $O
b() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie "$@" > $O/$tag.json 2> $O/$tag.err || exit $?; }
for rep in 1 2; do
  for sp in 0 5 15 30 60; do
    b f1d4_s${sp}_$rep --batch 1 --inflight 4 --set order_split=$sp
    b f8d2_s${sp}_$rep --batch 8 --inflight 2 --set order_split=$sp
  done
  b f8d2_nohf_$rep --batch 8 --inflight 2 --set heavy_first=0
  b f8d4_s15_$rep --batch 8 --inflight 4 --set order_split=15
done
echo done > $O/done.txt
