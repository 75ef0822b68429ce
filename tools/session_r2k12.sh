#!/bin/bash
# Session r2k12 (one GPU): round-2 closing evidence on HEAD — every GPU test,
# smoke, bench at the driver's 20 steps, rocprof, PMC passes A-C, configs 4/5/6.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2k12}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/gpu_session.sh "$TAG" test smoke bench prof || exit $?
PMC_PASSES="A B C" bash tools/pmc.sh "${TAG}_pmc" || exit $?
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
for a in "4 50" "5 20" "6 200"; do
  set -- $a
  st "start cfg$1"
  timeout -k 10 300 python bench.py --config $1 --steps $2 --warmup 3 --no-cpu-baseline > "$OUT/bench_cfg$1.json" \
    2> "$OUT/bench_cfg$1.err"; rc=$?; st "end rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
st "r2k12 done"
