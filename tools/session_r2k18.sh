#!/bin/bash
# Session r2k18 (one GPU): the async readback split over two copy streams
# (option copy_streams): its GPU tests, then tools/pipeline_bench.py (4 slots,
# 1 vs 2 copy streams, 400 frames each, two rounds).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2k18}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
st "start pytest"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rA -k "async or hip_engine" --timeout 120 \
  --timeout-method thread > "$OUT/pytest_async.log" 2>&1; rc=$?; st "end pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  st "start pipeline $rep"
  timeout -k 10 300 python tools/pipeline_bench.py --slots 4 --copy-streams 1,2 --frames 400 >> "$OUT/pipeline.jsonl" \
    2>> "$OUT/pipeline.err"; rc=$?; st "end rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
st "session done"
