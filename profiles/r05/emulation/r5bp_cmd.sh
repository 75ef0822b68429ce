set -u
O=gpurun_out/r5bp; mkdir -p $O
for rep in 1 2; do
  bash tools/emulate.sh $O/emu def_rep$rep 2 "1" --steps 20 --warmup 5 || exit $?
  bash tools/emulate.sh $O/emu lpoff_rep$rep 2 "1" --steps 20 --warmup 5 --last-pieces off || exit $?
  bash tools/emulate.sh $O/emu oldsettle_rep$rep 2 "1" --steps 20 --warmup 5 --settle-s 0.4 --settle-max 100 || exit $?
  bash tools/emulate.sh $O/emu both_rep$rep 2 "1" --steps 20 --warmup 5 --settle-s 0.4 --settle-max 100 --last-pieces off || exit $?
done
