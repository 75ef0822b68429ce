#!/bin/bash
# Session r2k14 (one GPU): frames in flight per config at N = 1 (bench.py
# --inflight): config 5 (the 1M-triangle scene, HBM-bound) at 1/2/3/4/6 and
# config 6 at 3/4/6, two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2k14}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
ab() { local tag=$1; shift; st "start $tag"; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" \
  > "$OUT/$tag.json" 2>> "$OUT/ab.err"; local rc=$?; st "end rc=$rc"; return $rc; }
for rep in 1 2; do
  for d in 1 2 3 4 6; do ab c5_d${d}_$rep --config 5 --steps 24 --warmup 3 --inflight $d || exit $?; done
  for d in 3 4 6; do ab c6_d${d}_$rep --config 6 --steps 200 --inflight $d || exit $?; done
done
st "session done"
