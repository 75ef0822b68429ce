#!/bin/bash
# Session r2k2 (one GPU): where the N > 1 exchange path loses time at world
# size 1 over RCCL (bench.py with BENCH_FORCE_DIST=1 ran 0.385 ms per frame
# of device time vs 0.318 for whole frames, r2k1): a kernel trace of it, and
# bench variants (frames in flight / exchange batch).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2k2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
export BENCH_FORCE_DIST=1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1
st "start prof"
MASTER_PORT=$((29500 + RANDOM % 1000)) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$OUT/prof" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-single \
  > "$OUT/prof_bench.json" 2> "$OUT/prof.err"; rc=$?; st "end prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
for arm in "--steps 20" "--steps 200" "--steps 200 --inflight 8" "--steps 200 --band 1080"; do
  st "start $arm"
  MASTER_PORT=$((29500 + RANDOM % 1000)) timeout -k 10 300 python3 bench.py --gpus 1 --warmup 5 --no-cpu-baseline \
    $arm >> "$OUT/arms.jsonl" 2>> "$OUT/arms.err"; rc=$?; st "end rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
st "session done"
