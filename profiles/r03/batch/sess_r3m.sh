# r3m: why do launches of several frames trace slower per frame than one
# frame per launch (N = 1, whole frames of config 3, 200 steps)?
set -u
O=gpurun_out/r3m
mkdir -p $O
b() { local tag=$1; shift; RTAMD_DEBUG_ORDER=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie "$@" > $O/$tag.json 2> $O/$tag.err || exit $?; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20_pcie.json 2> $O/bench20_pcie.err || exit $?
b f1d4 --batch 1 --inflight 4
b f2d2 --batch 2 --inflight 2
b f4d2 --batch 4 --inflight 2
b f8d2 --batch 8 --inflight 2
b f8d4 --batch 8 --inflight 4
b f8d1 --batch 8 --inflight 1
b f8d2_nohf --batch 8 --inflight 2 --set heavy_first=0
b f8d2_nohpx --batch 8 --inflight 2 --set heavy_pixels=0
b f1d4_nohf --batch 1 --inflight 4 --set heavy_first=0
b f1d1 --batch 1 --inflight 1
b f1d2 --batch 1 --inflight 2
b f1d8 --batch 1 --inflight 8
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_f8d2 -o run -- \
  python3 bench.py --batch 8 --inflight 2 --steps 40 --warmup 5 --no-cpu-baseline --no-pcie > $O/prof_f8d2.json 2> $O/prof_f8d2.err || exit $?
echo done > $O/done.txt
