set -u
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcie > $O/base20.json 2> $O/base20.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie > $O/base200.json 2> $O/base200.err || exit $?
e() { local tag=$1 n=$2 r=$3; shift 3; bash tools/emulate.sh $O/emu $tag $n "$r" --warmup 5 "$@" || exit $?; }
BENCH_EMULATE_NOX=1 e nox_n1_bands_f8d4 1 0 --steps 200 --batch 8 --inflight 4 --exchange-every 32
BENCH_EMULATE_NOX=1 e nox_n1_bands_f1d4 1 0 --steps 200 --batch 1 --inflight 4 --exchange-every 4
BENCH_EMULATE_NOX=1 e nox_w 8 1 --steps 200
e w200 8 "0 1 7" --steps 200
e w20 8 "0 1 7" --steps 20
e w20 4 "0 1 3" --steps 20
e w20 2 "0 1" --steps 20
e w20_g16 8 "0 1" --steps 20 --exchange-every 16
e w200_d3 8 "1" --steps 200 --inflight 3
e w200_d6 8 "1" --steps 200 --inflight 6
e w200_rw9 8 "0 1" --steps 200 --root-weight 0.9
e s20 8 "0 1 7" --steps 20 --scaling strong
echo done > $O/done.txt
