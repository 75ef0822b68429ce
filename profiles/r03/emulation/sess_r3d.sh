set -u
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/base20.json 2> $O/base20.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie > $O/base200.json 2> $O/base200.err || exit $?
for N in 2 4 8; do
  bash tools/emulate.sh $O/emu def20 $N "0 1 $((N-1))" --steps 20 --warmup 5 || exit $?
done
bash tools/emulate.sh $O/emu def200 8 "0 1 7" --steps 200 --warmup 5 || exit $?
for fd in "1 4" "1 8" "2 4" "2 2" "4 2" "8 1"; do
  set -- $fd
  for rw in 0.7 1.0; do
    bash tools/emulate.sh $O/emu sw20_f$1_d$2_w$rw 8 "0 1" --steps 20 --warmup 5 --batch $1 --inflight $2 --root-weight $rw || exit $?
  done
done
echo done > $O/done.txt
