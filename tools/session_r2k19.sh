#!/bin/bash
# Session r2k19 (one GPU): two device frame buffers per async slot (a slot's
# next trace no longer waits for its last readback): the async GPU tests, then
# tools/pipeline_bench.py with 4 slots and 4 or 8 host frames pending, two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2k19}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
st "start pytest"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rA -k "async or hip_engine" --timeout 120 \
  --timeout-method thread > "$OUT/pytest_async.log" 2>&1; rc=$?; st "end pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  st "start pipeline $rep"
  timeout -k 10 300 python tools/pipeline_bench.py --slots 4 --depth 1,2 --frames 400 >> "$OUT/pipeline.jsonl" \
    2>> "$OUT/pipeline.err"; rc=$?; st "end rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
st "session done"
