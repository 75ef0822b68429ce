set -u
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie > $O/base200.json 2> $O/base200.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie --batch 2 --inflight 2 > $O/n1_f2d2.json 2> $O/n1_f2d2.err || exit $?
e() { local tag=$1 n=$2 r=$3; shift 3; bash tools/emulate.sh $O/emu $tag $n "$r" --steps 200 --warmup 5 "$@" || exit $?; }
BENCH_EMULATE_NOX=1 e nox_n1_bands_f1d4 1 0 --batch 1 --inflight 4
BENCH_EMULATE_NOX=1 e nox_w_f8d4 8 1
BENCH_EMULATE_NOX=1 e nox_w_f4d4 8 1 --batch 4
BENCH_EMULATE_NOX=1 e nox_w_f2d4 8 1 --batch 2
BENCH_EMULATE_NOX=1 e nox_s_f4d4 8 1 --scaling strong
e w_f8d4 8 "0 1"
e w_f8d4g32 8 "0 1" --exchange-every 32
e w_f4d4 8 "0 1" --batch 4
e s_f4d4 8 "0 1" --scaling strong
echo done > $O/done.txt
