#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r2e}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() { local name=$1 secs=$2; shift 2; echo "$(date +%T) start $name" >> "$OUT/status.txt"
  timeout -k 10 "$secs" "$@"; local rc=$?; echo "$(date +%T) end $name rc=$rc" >> "$OUT/status.txt"; return $rc; }
for v in "1 graph=1" "2 graph=1" "1 graph=0" "2 graph=0" "2 graph=0,heavy_stream=0" "2 graph=1,heavy_tiles=0" "1 graph=1,heavy_tiles=0"; do
  set -- $v
  step "if$1_$2" 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --inflight $1 --set $2 > "$OUT/bench_if$1_$2.json" 2>> "$OUT/bench.err" || exit $?
done
echo "$(date +%T) session done" >> "$OUT/status.txt"
