# r3dl: the weighted band deal run on over N frames (--deal rotate, one band
# list per frame) against the fixed deal, emulated rank by rank at the
# driver's 20 steps (twice, interleaved), and rehearsed (frames verified).
set -u
O=gpurun_out/r3dl
mkdir -p $O
b() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie "$@" > $O/$tag.json 2> $O/$tag.err || exit $?; }
e() { local tag=$1 n=$2 r=$3; shift 3; bash tools/emulate.sh $O/emu $tag $n "$r" --warmup 5 --steps 20 "$@" || exit $?; }
for rep in a b; do
  b base20_$rep --steps 20
  e rot$rep 8 "0 1 3 5 7" --deal rotate
  e fix$rep 8 "0 1 3 5 7" --deal fixed
done
e rot4 4 "0 1 3" --deal rotate
e fix4 4 "0 1 3" --deal fixed
bash tools/rehearse.sh $O/rehearse 8 bands --steps 20 --warmup 5 --deal rotate || exit $?
bash tools/rehearse.sh $O/rehearse 4 bands --steps 20 --warmup 5 --deal rotate --gather radiance || exit $?
echo done > $O/done.txt
