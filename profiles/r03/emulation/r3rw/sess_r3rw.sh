# r3rw: rank 0's weight with dealt bands at N = 8 (0.7 / 0.8 / 0.9), ranks 0
# and 1 (the senders are even), three interleaved runs at the driver's 20 steps.
set -u
O=gpurun_out/r3rw
mkdir -p $O
e() { local tag=$1 n=$2 r=$3; shift 3; bash tools/emulate.sh $O/emu $tag $n "$r" --warmup 5 --steps 20 "$@" || exit $?; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie --steps 20 > $O/base20.json 2> $O/base20.err || exit $?
for rep in a b c; do
  for w in 0.7 0.8 0.9; do
    e w${w}$rep 8 "0 1" --root-weight $w
  done
done
echo done > $O/done.txt
