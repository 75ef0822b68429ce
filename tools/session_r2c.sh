#!/bin/bash
# bench at N=1 (default and inflight 2), strong-scaling model with inflight,
# 2-rank rehearsal of the bands default (inflight 2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r2c}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() { local name=$1 secs=$2; shift 2; echo "$(date +%T) start $name" >> "$OUT/status.txt"
  timeout -k 10 "$secs" "$@"; local rc=$?; echo "$(date +%T) end $name rc=$rc" >> "$OUT/status.txt"; return $rc; }
step bench 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
step bench_if2 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --inflight 2 > "$OUT/bench_if2.json" 2> "$OUT/bench_if2.err" || exit $?
step bench_if3 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --inflight 3 > "$OUT/bench_if3.json" 2> "$OUT/bench_if3.err" || exit $?
TAG=$TAG BACKENDS=gloo NPROC=2 PARTS=bands step rehearsal2 600 bash tools/dist_rehearsal.sh || exit $?
echo "$(date +%T) session done" >> "$OUT/status.txt"
