# r3t: bench.py's final N > 1 defaults (weak scaling, weighted bands, rank 0
# weight 0.9 / 0.85 / 0.8 at N = 2 / 4 / 8, order_split 15, exchange every 4
# launches) emulated rank by rank at the driver's 20 steps (twice) and at 200,
# and rehearsed with gloo ranks sharing the GPU (frames verified).
set -u
O=gpurun_out/r3t
mkdir -p $O
b() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie "$@" > $O/$tag.json 2> $O/$tag.err || exit $?; }
e() { local tag=$1 n=$2 r=$3; shift 3; bash tools/emulate.sh $O/emu $tag $n "$r" --warmup 5 "$@" || exit $?; }
for rep in a b; do
  b base20_$rep --steps 20
  e d20$rep 8 "0 1 3 5 7" --steps 20
  e d20$rep 4 "0 1 3" --steps 20
  e d20$rep 2 "0 1" --steps 20
done
b base200
e d200 8 "0 1 7" --steps 200
e d200 2 "0 1" --steps 200
bash tools/rehearse.sh $O/rehearse 8 bands --steps 20 --warmup 5 || exit $?
bash tools/rehearse.sh $O/rehearse 4 bands --steps 20 --warmup 5 --gather radiance || exit $?
bash tools/rehearse.sh $O/rehearse 2 bands --steps 20 --warmup 5 || exit $?
bash tools/rehearse.sh $O/rehearse 8 pieces --steps 20 --warmup 5 --root-weight 0.7 || exit $?
bash tools/rehearse.sh $O/rehearse 4 tiles --steps 20 --warmup 5 --gather radiance || exit $?
# pieces at 20 steps, every rank: learned order quality (learn_alone) and order_split
e p20alone 8 "0 1 2 3 4 5 6 7" --steps 20 --partition pieces --root-weight 0.7 --set order_split=15,learn_alone=1
e p20s40 8 "1 3 5" --steps 20 --partition pieces --root-weight 0.7 --set order_split=40
echo done > $O/done.txt
