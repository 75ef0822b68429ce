set -u
O=gpurun_out/r5bg; mkdir -p $O
BENCH_SHARE_GPU=1 BENCH_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 8 --steps 4 --warmup 1 --span-cut frames --no-single > $O/spawn8_frames.json 2> $O/spawn8_frames.err || exit $?
BENCH_SHARE_GPU=1 BENCH_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 3 --steps 8 --warmup 2 --span-cut frames --wire rgb > $O/spawn3_frames.json 2> $O/spawn3_frames.err || exit $?
for rep in 1 2; do
  bash tools/emulate.sh $O/emu fr_rep$rep 8 "0 1 2" --steps 20 --warmup 5 --span-cut frames || exit $?
  bash tools/emulate.sh $O/emu bd_rep$rep 8 "0 1" --steps 20 --warmup 5 || exit $?
  bash tools/emulate.sh $O/emu fr_rep$rep 4 "0 1" --steps 20 --warmup 5 --span-cut frames || exit $?
  bash tools/emulate.sh $O/emu bd_rep$rep 4 "0 1" --steps 20 --warmup 5 || exit $?
done
