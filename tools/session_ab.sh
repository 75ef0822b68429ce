#!/bin/bash
# Generic A/B: parity tests matching $KEXPR, then bench.py for each option set in
# $ARMS (space-separated; each arm is a --set string), $REPS times, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() { local name=$1 secs=$2; shift 2; echo "$(date +%T) start $name" >> "$OUT/status.txt"
  timeout -k 10 "$secs" "$@"; local rc=$?; echo "$(date +%T) end $name rc=$rc" >> "$OUT/status.txt"; return $rc; }
if [ -n "${KEXPR:-}" ]; then
  step pytest 600 python -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread -k "$KEXPR" > "$OUT/pytest_gpu.log" 2>&1 || exit $?
fi
for rep in $(seq 1 ${REPS:-2}); do
  i=0
  for arm in $ARMS; do
    i=$((i+1))
    step "bench_$i" 300 python bench.py --steps ${STEPS:-100} --warmup 5 --no-cpu-baseline --config ${CONFIG:-3} --set $arm > "$OUT/bench_a${i}_$rep.json" 2>> "$OUT/bench.err" || exit $?
  done
done
echo "$(date +%T) session done" >> "$OUT/status.txt"
