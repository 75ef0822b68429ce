#!/bin/bash
# Session r2k3 (one GPU): bench.py's N > 1 exchange path forced at world size
# 1 over RCCL (BENCH_FORCE_DIST=1), with and without the high-priority
# exchange streams (--exchange-priority), at the N = 1 and N = 8 frames in
# flight; then a kernel trace of the high-priority arm.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2k3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
export BENCH_FORCE_DIST=1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1
for rep in 1 2; do
  for arm in "--exchange-priority 0" "--exchange-priority 1" "--exchange-priority 0 --inflight 12" \
             "--exchange-priority 1 --inflight 12"; do
    st "start $arm rep $rep"
    MASTER_PORT=$((29500 + RANDOM % 1000)) timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 5 \
      --no-cpu-baseline $arm >> "$OUT/arms.jsonl" 2>> "$OUT/arms.err"; rc=$?; st "end rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
st "start prof"
MASTER_PORT=$((29500 + RANDOM % 1000)) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$OUT/prof" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-single \
  > "$OUT/prof_bench.json" 2> "$OUT/prof.err"; rc=$?; st "end prof rc=$rc"
st "session done"
