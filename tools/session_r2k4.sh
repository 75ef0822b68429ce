#!/bin/bash
# Session r2k4 (one GPU): the whole-frame parity tests of configs 3/4/5 under
# bench.py's setting, then rank 0 of N = 2/4/8 emulated with its exchange
# (tools/rank0_exchange_bench.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2k4}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
st "start pytest"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "bench_setting" --timeout 180 \
  --timeout-method thread > "$OUT/pytest_whole.log" 2>&1; rc=$?; st "end pytest rc=$rc"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
st "start rank0"
timeout -k 10 400 python tools/rank0_exchange_bench.py > "$OUT/rank0_exchange.jsonl" 2> "$OUT/rank0_exchange.err"
rc=$?; st "end rank0 rc=$rc"
st "session done"
