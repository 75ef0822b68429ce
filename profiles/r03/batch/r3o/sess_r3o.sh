# r3o: where does a weak-scaling rank's trace time go (pieces, N = 8, rank 1,
# 200 steps)?  Exchange off / heavy_first off / order_split / fewer frames per
# launch / fewer launches in flight; the lists path at N = 1; N = 1 batches with
# aligned phases.
set -u
O=gpurun_out/r3o
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie > $O/base200.json 2> $O/base200.err || exit $?
e() { local tag=$1 n=$2 r=$3; shift 3; bash tools/emulate.sh $O/emu $tag $n "$r" --warmup 5 --steps 200 "$@" || exit $?; }
e p 8 "1" --partition pieces
BENCH_EMULATE_NOX=1 e p_nox 8 "1" --partition pieces
e p_nohf 8 "1" --partition pieces --set heavy_first=0
e p_s15 8 "1" --partition pieces --set order_split=15
e p_d2 8 "1" --partition pieces --inflight 2
e p_d6 8 "1" --partition pieces --inflight 6
e p_f4 8 "1" --partition pieces --batch 4
e n1_f1 1 "0" --partition pieces --batch 1
e n1_f8 1 "0" --partition pieces --batch 8
b() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie "$@" > $O/$tag.json 2> $O/$tag.err || exit $?; }
b f8d2 --batch 8 --inflight 2
b f8d4 --batch 8 --inflight 4
b f8d2_nohf --batch 8 --inflight 2 --set heavy_first=0

# weighted pieces: rank 0's piece smaller (its receive + assembly)
e pw9 8 "0 1" --partition pieces --root-weight 0.9
e pw8 8 "0 1" --partition pieces --root-weight 0.8
e pw8_20 8 "0 1" --partition pieces --root-weight 0.8 --steps 20
e b_20 8 "0 1" --partition bands --steps 20
echo done2 > $O/done2.txt
