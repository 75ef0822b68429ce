#!/bin/bash
# Round-2 session: parity tests (new heavy-cap test), bench, strong-scaling
# model (rank shares on one GPU), 2- and 4-rank rehearsals with HEAD's bench.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r2b}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() { local name=$1 secs=$2; shift 2; echo "$(date +%T) start $name" >> "$OUT/status.txt"
  timeout -k 10 "$secs" "$@"; local rc=$?; echo "$(date +%T) end $name rc=$rc" >> "$OUT/status.txt"; return $rc; }
step pytest 600 python -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit $?
step bench 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
step share 300 python tools/rank_share_bench.py > "$OUT/rank_share.jsonl" 2> "$OUT/rank_share.err" || exit $?
TAG=$TAG BACKENDS=gloo NPROC=2 step rehearsal2 600 bash tools/dist_rehearsal.sh || exit $?
TAG=$TAG BACKENDS=gloo NPROC=4 step rehearsal4 600 bash tools/dist_rehearsal.sh || exit $?
echo "$(date +%T) session done" >> "$OUT/status.txt"
