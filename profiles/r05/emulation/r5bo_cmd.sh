set -u
O=gpurun_out/r5bo; mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench200.json 2> $O/bench200.err || exit $?
BENCH_SHARE_GPU=1 BENCH_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/spawn2.json 2> $O/spawn2.err || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcie --no-lanes > $O/n1_a.json 2> $O/n1_a.err || exit $?
bash tools/emulate.sh $O/emu s20 8 "0 1 7" --steps 20 --warmup 5 || exit $?
bash tools/emulate.sh $O/emu s20 4 "0 1" --steps 20 --warmup 5 || exit $?
bash tools/emulate.sh $O/emu s20 2 "0 1" --steps 20 --warmup 5 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcie --no-lanes > $O/n1_b.json 2> $O/n1_b.err || exit $?
