set -u
O=gpurun_out/r5bf; mkdir -p $O
for rep in 1 2; do
  bash tools/emulate.sh $O/emu def_rep$rep 8 "1 0" --steps 20 --warmup 5 || exit $?
  bash tools/emulate.sh $O/emu if6_rep$rep 8 "1 0" --steps 20 --warmup 5 --inflight 6 || exit $?
  bash tools/emulate.sh $O/emu g80_rep$rep 8 "1 0" --steps 20 --warmup 5 --exchange-every 80 || exit $?
done
