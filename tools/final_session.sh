#!/bin/bash
# Round-end evidence on one GPU: parity tests, smoke, bench (+rocprof), PMC
# passes, config-5 bench, PCIe-inclusive pipeline and frames-in-flight runs.
# Every GPU step has its own limit; a failure ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/gpu_session.sh "$TAG" test smoke bench prof || exit $?
bash tools/pmc.sh "${TAG}_pmc" || exit $?
step() { local name=$1 secs=$2; shift 2; echo "$(date +%T) start $name" >> "$OUT/status.txt"
  timeout -k 10 "$secs" "$@"; local rc=$?; echo "$(date +%T) end $name rc=$rc" >> "$OUT/status.txt"; return $rc; }
step cfg5 300 python bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_cfg5.json" 2> "$OUT/bench_cfg5.err" || exit $?
step pipeline 300 python tools/pipeline_bench.py > "$OUT/pipeline.jsonl" 2> "$OUT/pipeline.err" || exit $?
step inflight 300 python tools/inflight_bench.py > "$OUT/inflight.jsonl" 2> "$OUT/inflight.err" || exit $?
echo "$(date +%T) final session done" >> "$OUT/status.txt"
