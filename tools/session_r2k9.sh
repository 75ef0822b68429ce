#!/bin/bash
# Session r2k9 (one GPU): evidence on HEAD — the GPU tests, smoke, bench
# (driver's 20 steps) and rocprof; bench's N > 1 path forced at N = 1 over
# RCCL; 2- and 4-rank gloo rehearsals of the default partition.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2k9}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/gpu_session.sh "$TAG" test smoke bench prof || exit $?
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
st "start forced"
BENCH_FORCE_DIST=1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29500 + RANDOM % 1000)) \
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
  > "$OUT/bench_forced_dist_nccl_n1.json" 2> "$OUT/forced.err"; rc=$?; st "end rc=$rc"; [ $rc -ne 0 ] && exit $rc
TAG=$TAG/rehearsal BACKENDS=gloo NPROC=2 PARTS="bands" timeout -k 10 400 bash tools/dist_rehearsal.sh || exit $?
TAG=$TAG/rehearsal BACKENDS=gloo NPROC=4 PARTS="bands" timeout -k 10 400 bash tools/dist_rehearsal.sh || exit $?
st "r2k9 done"
