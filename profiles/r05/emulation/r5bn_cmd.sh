set -u
O=gpurun_out/r5bn; mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcie --no-lanes > $O/def_rep$rep.json 2> $O/def_rep$rep.err || exit $?
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcie --no-lanes --settle-s 1 --settle-max 1000 > $O/s1_rep$rep.json 2> $O/s1_rep$rep.err || exit $?
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcie --no-lanes --settle-s 3 --settle-max 3000 > $O/s3_rep$rep.json 2> $O/s3_rep$rep.err || exit $?
done
