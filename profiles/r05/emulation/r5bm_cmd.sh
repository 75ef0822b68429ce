set -u
O=gpurun_out/r5bm; mkdir -p $O
BENCH_SHARE_GPU=1 BENCH_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/spawn2.json 2> $O/spawn2.err || exit $?
for rep in 1 2; do
  bash tools/emulate.sh $O/emu def_rep$rep 8 "0 1" --steps 20 --warmup 5 || exit $?
  bash tools/emulate.sh $O/emu settle_rep$rep 8 "1" --steps 20 --warmup 5 --settle-s 3 --settle-max 2000 || exit $?
  bash tools/emulate.sh $O/emu def_rep$rep 4 "0 1" --steps 20 --warmup 5 || exit $?
  bash tools/emulate.sh $O/emu def_rep$rep 2 "0 1" --steps 20 --warmup 5 || exit $?
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcie --no-lanes > $O/n1.json 2> $O/n1.err || exit $?
