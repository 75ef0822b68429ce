# r3p: order_split with the weighted pieces and the weighted bands (N = 8
# emulated), and at N = 1.
set -u
O=gpurun_out/r3p
mkdir -p $O
b() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie "$@" > $O/$tag.json 2> $O/$tag.err || exit $?; }
e() { local tag=$1 n=$2 r=$3; shift 3; bash tools/emulate.sh $O/emu $tag $n "$r" --warmup 5 "$@" || exit $?; }
b base200
e pw8s15 8 "0 1" --steps 200 --partition pieces --root-weight 0.8 --set order_split=15
e pw9s15 8 "0 1" --steps 200 --partition pieces --root-weight 0.9 --set order_split=15
e pw8s30 8 "0 1" --steps 200 --partition pieces --root-weight 0.8 --set order_split=30
e pw8s5 8 "0 1" --steps 200 --partition pieces --root-weight 0.8 --set order_split=5
e bs15 8 "0 1" --steps 200 --partition bands --set order_split=15
e pw8s15_20 8 "0 1 7" --steps 20 --partition pieces --root-weight 0.8 --set order_split=15
e bs15_20 8 "0 1" --steps 20 --partition bands --set order_split=15
e pw85s15_20 4 "0 1" --steps 20 --partition pieces --root-weight 0.85 --set order_split=15
e ps15_20 2 "0 1" --steps 20 --partition pieces --set order_split=15
for rep in 1 2; do
  b f1d4_s0_$rep --set order_split=0
  b f1d4_s5_$rep --set order_split=5
  b f1d4_s15_$rep --set order_split=15
  b f1d4_s0_20_$rep --set order_split=0 --steps 20
  b f1d4_s15_20_$rep --set order_split=15 --steps 20
done
echo done > $O/done.txt
