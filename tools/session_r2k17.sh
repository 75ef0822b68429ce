#!/bin/bash
# Session r2k17 (one GPU): PMC passes A and H (instruction counts, TA busy)
# for walks 2 (default), 5 (scalar loads) and 14 (LDS-DMA) on config 3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2k17}
for w in 2 5 14; do
  BENCH_ARGS="--set walk=$w" PMC_PASSES="A H" bash tools/pmc.sh "${TAG}_w$w" || exit $?
done
