#!/bin/bash
# Round 6: the A/Bs session f could not run (its variant builds predated the
# runs entry point): the thin-triangle margins against round 5's fixed factor
# (RT_THIN_MARGIN=0) on configs 3 and 5, and the trace schedule against the
# compiler's default.  Each GPU step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
chk() { local rc=$1; st "rc=$rc"; if [ "$rc" -ne 0 ]; then st "abort"; exit "$rc"; fi; }
L=3d-ray-tracer-vulkan_amd/lib
st "ab margin c3"; REPS=3 bash tools/ab_lib.sh "$OUT/ab3" "--steps 200 --warmup 5" $L/librtamd.so $L/variants/librtamd_nomargin.so; chk $?
st "ab margin c5"; REPS=2 bash tools/ab_lib.sh "$OUT/ab5" "--config 5 --steps 20 --warmup 3" $L/librtamd.so $L/variants/librtamd_nomargin.so; chk $?
st "ab sched c3"; REPS=3 bash tools/ab_lib.sh "$OUT/absched" "--steps 200 --warmup 5" $L/librtamd.so $L/variants/librtamd_defsched.so; chk $?
st done
