#!/bin/bash
# Session r2k8 (one GPU): exchange-ring depth (2 vs 4 batches) for the
# emulated rank 0 (receiver) and rank 1 (sender) at N = 8, blocks (root_share
# 0.6 and 1) and bands, trace-only arms beside; two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2k8}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
em() { st "start em $*"; timeout -k 10 400 python tools/rank0_exchange_bench.py "$@" >> "$OUT/emulate.jsonl" \
  2>> "$OUT/emulate.err"; local rc=$?; st "end rc=$rc"; return $rc; }
for rep in 1 2; do
  for ring in 2 4; do
    em --ranks 8 --rank 0 --ring $ring --arms bands:0:0,bands:1:1,blocks:0:0:0.6,blocks:1:1:0.6,blocks:1:1:1.0 || exit $?
    em --ranks 8 --rank 1 --ring $ring --arms blocks:0:0:0.6,blocks:1:1:0.6 || exit $?
  done
done
st "session done"
