#!/bin/bash
# Session r2k11 (one GPU): walk 14 (LDS-DMA fetches on wave-uniform steps) on the
# round-2 default: its parity tests, then an A/B against walk 2 (bench.py,
# config 3 x3 at 200 steps, config 6 x2, config 5 x1, interleaved).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2k11}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
st "start pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rA -k "walk or schedules or bench_setting" \
  --timeout 180 --timeout-method thread > "$OUT/pytest_walk5.log" 2>&1; rc=$?; st "end pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
ab() { local tag=$1; shift; st "start $tag"; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$OUT/$tag.json" \
  2>> "$OUT/ab.err"; local rc=$?; st "end rc=$rc"; return $rc; }
for rep in 1 2 3; do
  ab c3_w2_$rep --steps 200 || exit $?
  ab c3_w14_$rep --steps 200 --set walk=14 || exit $?
done
for rep in 1 2; do
  ab c6_w2_$rep --config 6 --steps 200 || exit $?
  ab c6_w14_$rep --config 6 --steps 200 --set walk=14 || exit $?
done
ab c5_w2_1 --config 5 --steps 20 --warmup 3 || exit $?
ab c5_w14_1 --config 5 --steps 20 --warmup 3 --set walk=14 || exit $?
st "session done"
