# r3s: pieces (w 0.7 / 0.75 / 1.0) against weighted bands at the driver's 20
# steps, on one box, twice, every rank that differs (N = 8 / 4 / 2 emulated).
set -u
O=gpurun_out/r3s
mkdir -p $O
b() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie "$@" > $O/$tag.json 2> $O/$tag.err || exit $?; }
e() { local tag=$1 n=$2 r=$3; shift 3; bash tools/emulate.sh $O/emu $tag $n "$r" --warmup 5 --steps 20 --set order_split=15 "$@" || exit $?; }
for rep in a b; do
  b base20_$rep --steps 20
  e p8$rep 8 "0 1 3 5 7" --partition pieces --root-weight 0.7
  e b8$rep 8 "0 1 3 5 7" --partition bands --root-weight 0.7
  e p4$rep 4 "0 1 3" --partition pieces --root-weight 0.75
  e b4$rep 4 "0 1 3" --partition bands --root-weight 0.85
  e p2$rep 2 "0 1" --partition pieces --root-weight 1.0
  e b2$rep 2 "0 1" --partition bands --root-weight 1.0
done
echo done > $O/done.txt
