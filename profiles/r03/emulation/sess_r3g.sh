set -u
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie > $O/base200.json 2> $O/base200.err || exit $?
e() { local tag=$1 n=$2 r=$3; shift 3; BENCH_EMULATE_NOX=1 bash tools/emulate.sh $O/emu $tag $n "$r" --steps 200 --warmup 5 "$@" || exit $?; }
e n1_bands_f1d4 1 0 --batch 1 --inflight 4
e n1_bands_f2d2 1 0 --batch 2 --inflight 2
e n1_bands_f8d2 1 0 --batch 8 --inflight 2
e w_f8d4g8 8 1
e w_f8d4g32 8 1 --exchange-every 32
e w_f8d8g8 8 1 --inflight 8
e w_f4d4 8 1 --batch 4
e w_f2d4 8 1 --batch 2
e w_f2d8 8 1 --batch 2 --inflight 8
e w_f1d8 8 1 --batch 1 --inflight 8
e s_f4d4 8 1 --scaling strong
e s_f2d4 8 1 --scaling strong --batch 2
echo done > $O/done.txt
