#!/bin/bash
# A/B of bench.py between this tree and an older one checked out (and built)
# under build_ab/old (git worktree add build_ab/old <commit>), interleaved.
# Usage: tools/ab_old_new.sh OUTDIR [ROUNDS] [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; ROUNDS=${2:-3}; shift 2 || shift $#
mkdir -p "$OUT"
for i in $(seq 1 "$ROUNDS"); do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie "$@" > "$OUT/new_$i.json" 2> "$OUT/new_$i.err" || exit $?
  (cd build_ab/old && timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "../../$OUT/old_$i.json" 2> "../../$OUT/old_$i.err") || exit $?
done
