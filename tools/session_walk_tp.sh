#!/bin/bash
# Throughput-bound comparison of walks: config 5 bench and config 3 with
# frames in flight (tools/inflight_bench.py), per RTAMD_WALK value.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-wtp}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() { local name=$1 secs=$2; shift 2; echo "$(date +%T) start $name" >> "$OUT/status.txt"
  timeout -k 10 "$secs" "$@"; local rc=$?; echo "$(date +%T) end $name rc=$rc" >> "$OUT/status.txt"; return $rc; }
for w in ${WALKS:-2 5}; do
  RTAMD_WALK=$w step "cfg5_w$w" 300 python bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/cfg5_w$w.json" 2>> "$OUT/err.txt" || exit $?
  RTAMD_WALK=$w step "inflight_w$w" 300 python tools/inflight_bench.py --streams 1,3 --frames 60 > "$OUT/inflight_w$w.jsonl" 2>> "$OUT/err.txt" || exit $?
done
echo "$(date +%T) session done" >> "$OUT/status.txt"
