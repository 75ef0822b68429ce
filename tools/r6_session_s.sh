#!/bin/bash
# Round 6: the format-0 walk starts inside the root (RT_ROOT_ENTER): GPU
# suite and smoke, then an A/B against the previous tree (prev), configs 3
# and 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
chk() { local rc=$1; st "rc=$rc"; if [ "$rc" -ne 0 ]; then st "abort"; exit "$rc"; fi; }
L=3d-ray-tracer-vulkan_amd/lib
st "pytest"; timeout -k 10 1200 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1; chk $?
st "smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; chk $?
V="$L/librtamd.so $L/variants/librtamd_prev.so"
st "ab c3"; REPS=3 bash tools/ab_lib.sh "$OUT/ab3" "--steps 200 --warmup 5" $V; chk $?
st "ab c5"; REPS=2 bash tools/ab_lib.sh "$OUT/ab5" "--config 5 --steps 20 --warmup 3" $V; chk $?
st done
