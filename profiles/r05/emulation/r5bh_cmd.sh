set -u
O=gpurun_out/r5bh; mkdir -p $O
for rep in 1 2; do
  bash tools/emulate.sh $O/emu lag1_rep$rep 8 "1" --steps 20 --warmup 5 || exit $?
  bash tools/emulate.sh $O/emu lag2_rep$rep 8 "1" --steps 20 --warmup 5 --send-lag 2 || exit $?
  bash tools/emulate.sh $O/emu inf8_rep$rep 8 "1" --steps 20 --warmup 5 --inflight 8 || exit $?
done
