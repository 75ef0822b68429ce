set -u
O=gpurun_out/r5bs; mkdir -p $O
for rep in 1 2 3; do
  bash tools/emulate.sh $O/emu on_rep$rep 2 "1" --steps 20 --warmup 5 || exit $?
  bash tools/emulate.sh $O/emu off_rep$rep 2 "1" --steps 20 --warmup 5 --last-pieces off || exit $?
done
