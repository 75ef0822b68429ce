set -u
O=gpurun_out/r5bb; mkdir -p $O
export BENCH_SHARE_GPU=1 BENCH_DIST_BACKEND=gloo
timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/spawn2.json 2> $O/spawn2.err || exit $?
timeout -k 10 300 python bench.py --gpus 4 --steps 8 --warmup 2 --wire rgb > $O/spawn4_rgb.json 2> $O/spawn4_rgb.err || exit $?
timeout -k 10 300 python bench.py --gpus 3 --steps 6 --warmup 3 --last-pieces off > $O/spawn3_off.json 2> $O/spawn3_off.err || exit $?
unset BENCH_SHARE_GPU BENCH_DIST_BACKEND
for rep in 1 2; do
  for lp in on off; do
    bash tools/emulate.sh $O/emu lp${lp}_rep$rep 8 "0 1" --steps 20 --warmup 5 --last-pieces $lp || exit $?
  done
done
