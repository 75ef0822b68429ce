#!/bin/bash
# Session r2k5 (one GPU): rank 0 of N = 2/4/8 emulated for the interleaved
# bands and the rotating blocks partitions (tools/rank0_exchange_bench.py),
# then bench.py's blocks path forced at world size 1 over RCCL.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2k5}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
st "start rank0"
timeout -k 10 500 python tools/rank0_exchange_bench.py > "$OUT/rank0_exchange.jsonl" 2> "$OUT/rank0_exchange.err"
rc=$?; st "end rank0 rc=$rc"; [ $rc -ne 0 ] && exit $rc
export BENCH_FORCE_DIST=1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1
for arm in "--partition blocks --steps 20" "--partition blocks --steps 200" "--partition bands --steps 200"; do
  st "start $arm"
  MASTER_PORT=$((29500 + RANDOM % 1000)) timeout -k 10 300 python3 bench.py --gpus 1 --warmup 5 --no-cpu-baseline \
    $arm >> "$OUT/forced.jsonl" 2>> "$OUT/forced.err"; rc=$?; st "end rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
st "session done"
# bench.py's N > 1 paths with ranks sharing the GPU (gloo; RCCL refuses two ranks on one GPU)
TAG=$TAG/rehearsal BACKENDS=gloo NPROC=2 PARTS="blocks bands" timeout -k 10 700 bash tools/dist_rehearsal.sh || exit $?
TAG=$TAG/rehearsal BACKENDS=gloo NPROC=4 PARTS="blocks" timeout -k 10 400 bash tools/dist_rehearsal.sh || exit $?
st "rehearsals done"
