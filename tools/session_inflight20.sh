#!/bin/bash
# bench.py at the driver's 20 steps / 5 warmup with D = $DS frames in flight,
# $REPS interleaved rounds (run-to-run spread of the short timed region).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r2if20}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in $(seq 1 ${REPS:-5}); do
  for d in ${DS:-4 6 8}; do
    timeout -k 10 120 python bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} --no-cpu-baseline --inflight $d ${BENCH_ARGS:-} \
      > "$OUT/d${d}_$r.json" 2> "$OUT/d${d}_$r.err" || exit $?
  done
done
echo done > "$OUT/done.txt"
