#!/bin/bash
# walk 3 (node pairs): parity tests, then A/B bench against walk 2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-w3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() { local name=$1 secs=$2; shift 2; echo "$(date +%T) start $name" >> "$OUT/status.txt"
  timeout -k 10 "$secs" "$@"; local rc=$?; echo "$(date +%T) end $name rc=$rc" >> "$OUT/status.txt"; return $rc; }
step pytest 600 python -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread -k "walk or schedules or unbalanced or spheres" > "$OUT/pytest_gpu.log" 2>&1 || exit $?
for rep in 1 2; do
for w in ${WALKS:-2 3}; do
  step "bench_w$w" 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --set walk=$w${EXTRA:+,$EXTRA} > "$OUT/bench_w${w}_$rep.json" 2>> "$OUT/bench.err" || exit $?
done
done
echo "$(date +%T) session done" >> "$OUT/status.txt"
