#!/bin/bash
# Round 6: per-step priority (RT_STEP_PRIO: 3 on the chain, 1 for triangle tests) against the walk at 2
# against this tree, configs 5 (fetch-bound) and 3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
chk() { local rc=$1; st "rc=$rc"; if [ "$rc" -ne 0 ]; then st "abort"; exit "$rc"; fi; }
L=3d-ray-tracer-vulkan_amd/lib
V="$L/librtamd.so $L/variants/librtamd_stepprio.so"
st "ab c5"; REPS=3 bash tools/ab_lib.sh "$OUT/ab5" "--config 5 --steps 20 --warmup 3" $V; chk $?
st "ab c3"; REPS=3 bash tools/ab_lib.sh "$OUT/ab3" "--steps 200 --warmup 5" $V; chk $?
st done
