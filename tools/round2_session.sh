#!/bin/bash
# Round-2 evidence on one GPU: parity tests, smoke, bench (+rocprof), PMC
# passes, configs 4/5/6, PCIe-inclusive pipeline, frames in flight, the
# strong-scaling model and 2-/4-rank rehearsals.  Every GPU step has its own
# limit; a failure ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export GPU_MAX_HW_QUEUES=16      # as bench.py sets it: one hardware queue per stream
TAG=${1:-r2final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/gpu_session.sh "$TAG" test smoke bench prof || exit $?
PMC_PASSES="A B C D E" bash tools/pmc.sh "${TAG}_pmc" || exit $?
step() { local name=$1 secs=$2; shift 2; echo "$(date +%T) start $name" >> "$OUT/status.txt"
  timeout -k 10 "$secs" "$@"; local rc=$?; echo "$(date +%T) end $name rc=$rc" >> "$OUT/status.txt"; return $rc; }
for c in 4 5 6; do
  step cfg$c 300 python bench.py --config $c --steps 50 --warmup 3 --no-cpu-baseline > "$OUT/bench_cfg$c.json" 2> "$OUT/bench_cfg$c.err" || exit $?
done
step pipeline 300 python tools/pipeline_bench.py > "$OUT/pipeline.jsonl" 2> "$OUT/pipeline.err" || exit $?
step inflight 300 python tools/inflight_bench.py > "$OUT/inflight.jsonl" 2> "$OUT/inflight.err" || exit $?
step share 300 python tools/share_inflight_bench.py --ranks 1,2,4,8 > "$OUT/share_inflight.jsonl" 2> "$OUT/share_inflight.err" || exit $?
TAG=$TAG BACKENDS=gloo NPROC=2 step rehearsal2 600 bash tools/dist_rehearsal.sh || exit $?
TAG=$TAG BACKENDS=gloo NPROC=4 PARTS=bands step rehearsal4 600 bash tools/dist_rehearsal.sh || exit $?
echo "$(date +%T) round2 session done" >> "$OUT/status.txt"
