#!/bin/bash
# Round 6: occupancy of the accel kernels: 8 (this tree), 7 and 6 waves per SIMD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
chk() { local rc=$1; st "rc=$rc"; if [ "$rc" -ne 0 ]; then st "abort"; exit "$rc"; fi; }
L=3d-ray-tracer-vulkan_amd/lib
V="$L/librtamd.so $L/variants/librtamd_wpe7.so $L/variants/librtamd_wpe6.so"
st "ab c3"; REPS=3 bash tools/ab_lib.sh "$OUT/ab3" "--steps 200 --warmup 5" $V; chk $?
st "ab c5"; REPS=2 bash tools/ab_lib.sh "$OUT/ab5" "--config 5 --steps 20 --warmup 3" $V; chk $?
st done
