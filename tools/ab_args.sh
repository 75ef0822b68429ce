#!/bin/bash
# A/B over bench.py argument sets: each arm is one quoted argument string in
# the array file $ARMS_FILE (one arm per line), $REPS interleaved rounds.
# Usage: ARMS_FILE=... REPS=2 bash tools/ab_args.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-abargs}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
mapfile -t ARMS < "$ARMS_FILE"
for rep in $(seq 1 ${REPS:-2}); do
  i=0
  for arm in "${ARMS[@]}"; do
    i=$((i+1))
    echo "$(date +%T) arm $i rep $rep: $arm" >> "$OUT/status.txt"
    timeout -k 10 300 python bench.py --steps ${STEPS:-100} --warmup 5 --no-cpu-baseline $arm \
      > "$OUT/a${i}_r$rep.json" 2>> "$OUT/bench.err" || exit $?
  done
done
echo "$(date +%T) done" >> "$OUT/status.txt"
