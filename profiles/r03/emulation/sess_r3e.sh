set -u
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcie > $O/base20.json 2> $O/base20.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie > $O/base200.json 2> $O/base200.err || exit $?
for N in 2 4 8; do
  bash tools/emulate.sh $O/emu weak20 $N "0 1 $((N-1))" --steps 20 --warmup 5 || exit $?
done
bash tools/emulate.sh $O/emu weak200 8 "0 1 7" --steps 200 --warmup 5 || exit $?
for rw in 0.5 0.7 0.85; do
  bash tools/emulate.sh $O/emu weak20_w$rw 8 "0 1" --steps 20 --warmup 5 --root-weight $rw || exit $?
done
for d in 2 3 6; do
  bash tools/emulate.sh $O/emu weak20_d$d 8 "0 1" --steps 20 --warmup 5 --inflight $d || exit $?
done
bash tools/emulate.sh $O/emu strong20 8 "0 1 7" --steps 20 --warmup 5 --scaling strong || exit $?
bash tools/emulate.sh $O/emu strong200 8 "0 1 7" --steps 200 --warmup 5 --scaling strong || exit $?
bash tools/rehearse.sh $O/rehearse 8 bands --steps 20 --warmup 5 || exit $?
bash tools/rehearse.sh $O/rehearse 4 bands --config 4 --steps 20 --warmup 5 --gather radiance || exit $?
echo done > $O/done.txt
