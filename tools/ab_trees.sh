#!/bin/bash
# A/B of whole trees (git worktrees under build_ab/, each built in place) by
# their own bench.py, interleaved: a bisection of a performance change.
# Usage: tools/ab_trees.sh OUTDIR ROUNDS "bench args" DIR [DIR ...]   (DIR "." = this tree)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$1; ROUNDS=$2; ARGS=$3; shift 3
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for d in "$@"; do
    name=$(basename "$(cd "$d" && pwd)")
    [ "$d" = "." ] && name=current
    echo "$(date +%T) $name round $r" >> "$OUT/status.txt"
    (cd "$d" && timeout -k 10 300 python bench.py --no-cpu-baseline $ARGS) > "$OUT/${name}_$r.json" 2>> "$OUT/bench.err" || exit $?
  done
done
