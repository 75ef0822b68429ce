set -u
O=gpurun_out/r3f
mkdir -p $O
b() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie "$@" > $O/$tag.json 2> $O/$tag.err || exit $?; }
b base200
b n1_f2_d2 --batch 2 --inflight 2
b n1_f2_d4 --batch 2 --inflight 4
b n1_f4_d1 --batch 4 --inflight 1
b n1_f4_d2 --batch 4 --inflight 2
b n1_f8_d1 --batch 8 --inflight 1
b n1_f8_d2 --batch 8 --inflight 2
b base200b
BENCH_EMULATE_NOX=1 bash tools/emulate.sh $O/emu nox 8 "0 1" --steps 200 --warmup 5 || exit $?
BENCH_EMULATE_NOX=1 bash tools/emulate.sh $O/emu nox_d2 8 "1" --steps 200 --warmup 5 --inflight 2 || exit $?
BENCH_EMULATE_NOX=1 bash tools/emulate.sh $O/emu nox_b16 8 "1" --steps 200 --warmup 5 --band 16 || exit $?
BENCH_EMULATE_NOX=1 bash tools/emulate.sh $O/emu nox_b64 8 "1" --steps 200 --warmup 5 --band 64 || exit $?
bash tools/emulate.sh $O/emu g32 8 "0 1" --steps 200 --warmup 5 --exchange-every 32 || exit $?
BENCH_EMULATE_NOX=1 bash tools/emulate.sh $O/emu nox_n2 2 "1" --steps 200 --warmup 5 || exit $?
echo done > $O/done.txt
