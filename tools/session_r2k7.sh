#!/bin/bash
# Session r2k7 (one GPU): the blocks partition's rank-0 share (root_share)
# emulated for rank 0 (receiver) and rank 1 (sender) at N = 4 and 8; bench's
# blocks path forced at world size 1 over RCCL; gloo rehearsals at N = 2, 4
# (ranks sharing the GPU) with frames verified.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2k7}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
em() { st "start em $*"; timeout -k 10 400 python tools/rank0_exchange_bench.py "$@" >> "$OUT/emulate.jsonl" \
  2>> "$OUT/emulate.err"; local rc=$?; st "end rc=$rc"; return $rc; }
em --ranks 8 --rank 0 --arms bands:1:1,blocks:1:1:1.0,blocks:1:1:0.6,blocks:1:1:0.4 || exit $?
em --ranks 8 --rank 1 --arms blocks:1:1:1.0,blocks:1:1:0.6,blocks:1:1:0.4 || exit $?
em --ranks 4 --rank 0 --arms bands:1:1,blocks:1:1:1.0,blocks:1:1:0.9,blocks:1:1:0.7 || exit $?
em --ranks 4 --rank 1 --arms blocks:1:1:1.0,blocks:1:1:0.9,blocks:1:1:0.7 || exit $?
export BENCH_FORCE_DIST=1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1
st "start forced"
MASTER_PORT=$((29500 + RANDOM % 1000)) timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 \
  --no-cpu-baseline > "$OUT/forced_blocks.json" 2> "$OUT/forced_blocks.err"; rc=$?; st "end rc=$rc"; [ $rc -ne 0 ] && exit $rc
unset BENCH_FORCE_DIST RANK LOCAL_RANK WORLD_SIZE MASTER_ADDR
TAG=$TAG/rehearsal BACKENDS=gloo NPROC=2 PARTS="blocks" timeout -k 10 400 bash tools/dist_rehearsal.sh || exit $?
TAG=$TAG/rehearsal BACKENDS=gloo NPROC=4 PARTS="blocks" timeout -k 10 400 bash tools/dist_rehearsal.sh || exit $?
st "session done"
