#!/bin/bash
# Evidence session + drain A/B: parity tests, smoke, bench (+rocprof), PMC,
# configs 4-6, then bench at the driver's 20 steps with --drain 0 / 1
# alternated.  Every GPU step has its own limit; a failure ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export GPU_MAX_HW_QUEUES=16
TAG=${1:-r2drain}
STEPS=${STEPS:-"test smoke bench prof"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() { local name=$1 secs=$2; shift 2; echo "$(date +%T) start $name" >> "$OUT/status.txt"
  timeout -k 10 "$secs" "$@"; local rc=$?; echo "$(date +%T) end $name rc=$rc" >> "$OUT/status.txt"; return $rc; }
if [ -n "$STEPS" ]; then bash tools/gpu_session.sh "$TAG" $STEPS || exit $?; fi
if [ -n "${PMC:-A B C}" ]; then PMC_PASSES="${PMC:-A B C}" bash tools/pmc.sh "${TAG}_pmc" || exit $?; fi
for c in ${CFGS:-4 5 6}; do
  n=50; [ "$c" = 5 ] && n=20
  step cfg$c 300 python bench.py --config $c --steps $n --warmup 3 --no-cpu-baseline \
      > "$OUT/bench_cfg$c.json" 2> "$OUT/bench_cfg$c.err" || exit $?
done
for r in ${AB_REPS:-1 2 3}; do
  for d in 0 1; do
    step drain${d}_$r 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --drain $d \
        > "$OUT/ab_drain${d}_$r.json" 2> "$OUT/ab_drain${d}_$r.err" || exit $?
  done
done
echo "$(date +%T) session done" >> "$OUT/status.txt"
