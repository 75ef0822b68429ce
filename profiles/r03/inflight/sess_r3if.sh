# r3if: launches in flight at N = 1 (D = 3 / 4 / 5 / 6) on the final build,
# interleaved twice at 200 steps and once at 20.
set -u
O=gpurun_out/r3if
mkdir -p $O
for rep in a b; do
  for d in 3 4 5 6; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie --steps 200 --inflight $d > $O/d${d}_$rep.json 2> $O/d${d}_$rep.err || exit $?
  done
done
for d in 3 4 5 6; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie --steps 20 --inflight $d > $O/d${d}_20.json 2> $O/d${d}_20.err || exit $?
done
echo done > $O/done.txt
