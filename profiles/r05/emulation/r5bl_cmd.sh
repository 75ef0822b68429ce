set -u
O=gpurun_out/r5bl; mkdir -p $O
for rep in 1 2; do
  bash tools/emulate.sh $O/emu def_rep$rep 8 "1" --steps 20 --warmup 5 || exit $?
  bash tools/emulate.sh $O/emu settle_rep$rep 8 "1" --steps 20 --warmup 5 --settle-s 3 --settle-max 2000 || exit $?
  bash tools/emulate.sh $O/emu warm_rep$rep 8 "1" --steps 20 --warmup 60 || exit $?
done
