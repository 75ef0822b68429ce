set -u
O=gpurun_out/r5be; mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcie --no-lanes > $O/n1.json 2> $O/n1.err || exit $?
for rep in 1 2; do
  bash tools/emulate.sh $O/emu os15_rep$rep 8 "1 0" --steps 20 --warmup 5 || exit $?
  bash tools/emulate.sh $O/emu os0_rep$rep 8 "1 0" --steps 20 --warmup 5 --set order_split=0 || exit $?
done
