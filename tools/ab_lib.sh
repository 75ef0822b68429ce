#!/bin/bash
# A/B of library builds (make variant NAME=x FLAGS=...): bench.py with
# RTAMD_LIB_PATH set to each build in turn, interleaved, $REPS rounds.
# Usage: REPS=3 bash tools/ab_lib.sh OUTDIR "bench args" lib1.so lib2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; ARGS=$2; shift 2
mkdir -p "$OUT"
for rep in $(seq 1 "${REPS:-3}"); do
  i=0
  for lib in "$@"; do
    i=$((i+1))
    echo "$(date +%T) lib $i ($lib) rep $rep" >> "$OUT/status.txt"
    RTAMD_LIB_PATH="$lib" timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie --no-lanes $ARGS \
      > "$OUT/l${i}_r$rep.json" 2>> "$OUT/bench.err" || exit $?
  done
done
