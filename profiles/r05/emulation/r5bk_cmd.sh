set -u
O=gpurun_out/r5bk; mkdir -p $O
RTAMD_DEBUG_PLAN=1 bash tools/emulate.sh $O/emu dbg 8 "1" --steps 20 --warmup 5 || exit $?
RTAMD_DEBUG_PLAN=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcie --no-lanes > $O/n1.json 2> $O/n1.err || exit $?
