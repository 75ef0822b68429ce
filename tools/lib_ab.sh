#!/bin/bash
# A/B of library builds: bench.py with RTAMD_LIB_PATH = each of $LIBS (paths
# relative to the repo; "default" = the in-tree lib), $REPS times, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-libab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in $(seq 1 ${REPS:-2}); do
  i=0
  for lib in $LIBS; do
    i=$((i+1))
    if [ "$lib" = default ]; then unset RTAMD_LIB_PATH; else export RTAMD_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 300 python bench.py --steps ${STEPS:-100} --warmup 5 --no-cpu-baseline --config ${CONFIG:-3} \
      > "$OUT/bench_a${i}_$rep.json" 2>> "$OUT/bench.err" || exit $?
  done
done
unset RTAMD_LIB_PATH
