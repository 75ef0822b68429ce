set -u
O=gpurun_out/r5bt; mkdir -p $O
for rep in 1 2 3; do
  bash tools/emulate.sh $O/emu host_rep$rep 2 "1" --steps 20 --warmup 5 || exit $?
  bash tools/emulate.sh $O/emu dev_rep$rep 2 "1" --steps 20 --warmup 5 --piece-wait device || exit $?
  bash tools/emulate.sh $O/emu off_rep$rep 2 "1" --steps 20 --warmup 5 --last-pieces off || exit $?
done
bash tools/emulate.sh $O/emu dev_rep1 8 "1" --steps 20 --warmup 5 --piece-wait device || exit $?
bash tools/emulate.sh $O/emu host_rep1 8 "1" --steps 20 --warmup 5 || exit $?
BENCH_SHARE_GPU=1 BENCH_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --piece-wait device > $O/spawn2_dev.json 2> $O/spawn2_dev.err || exit $?
