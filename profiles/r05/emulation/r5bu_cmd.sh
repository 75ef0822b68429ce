set -u
O=gpurun_out/r5bu; mkdir -p $O
for rep in 1 2 3; do
  bash tools/emulate.sh $O/emu p1_rep$rep 2 "1" --steps 20 --warmup 5 || exit $?
  bash tools/emulate.sh $O/emu p2_rep$rep 2 "1" --steps 20 --warmup 5 --exchange-priority 2 || exit $?
  bash tools/emulate.sh $O/emu off_rep$rep 2 "1" --steps 20 --warmup 5 --last-pieces off || exit $?
done
bash tools/emulate.sh $O/emu p2_rep1 8 "1 0" --steps 20 --warmup 5 --exchange-priority 2 || exit $?
bash tools/emulate.sh $O/emu p1_rep1 8 "1 0" --steps 20 --warmup 5 || exit $?
