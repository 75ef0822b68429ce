# r3e3: the final N > 1 defaults (dealt bands at N = 8) emulated rank by rank at 20 steps (twice) and rehearsed (frames verified).
set -u
O=gpurun_out/r3e3
mkdir -p $O
b() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie "$@" > $O/$tag.json 2> $O/$tag.err || exit $?; }
e() { local tag=$1 n=$2 r=$3; shift 3; bash tools/emulate.sh $O/emu $tag $n "$r" --warmup 5 "$@" || exit $?; }
for rep in a b; do
  b base20_$rep --steps 20
  e d20$rep 8 "0 1 3 5 7" --steps 20
  e d20$rep 4 "0 1 3" --steps 20
  e d20$rep 2 "0 1" --steps 20
done
bash tools/rehearse.sh $O/rehearse 8 bands --steps 20 --warmup 5 || exit $?
bash tools/rehearse.sh $O/rehearse 4 bands --steps 20 --warmup 5 --gather radiance || exit $?
bash tools/rehearse.sh $O/rehearse 2 bands --steps 20 --warmup 5 || exit $?
bash tools/rehearse.sh $O/rehearse 8 pieces --steps 20 --warmup 5 --root-weight 0.7 || exit $?
bash tools/rehearse.sh $O/rehearse 4 tiles --steps 20 --warmup 5 --gather radiance || exit $?
echo done > $O/done.txt
