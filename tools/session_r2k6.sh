#!/bin/bash
# Session r2k6 (one GPU): rank 0 of N = 4 / 8 emulated, bands vs blocks, the
# blocks receive emulated as one RCCL copy of its volume; two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2k6}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
for rep in 1 2; do
  st "start rank0 $rep"
  timeout -k 10 400 python tools/rank0_exchange_bench.py --ranks 4,8 >> "$OUT/rank0_exchange.jsonl" 2>> "$OUT/rank0_exchange.err"
  rc=$?; st "end rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
st "session done"
