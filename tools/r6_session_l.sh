#!/bin/bash
# Round 6: the accel records' packed-pair slot layout (lo.xy hi.xy | lo.z hi.z
# link w7): 3 + 3 packed slab instructions per step.
# GPU suite and smoke, bench, then an A/B on one box
# against the previous tree (bytes) and without the forced bit, configs 3 and 5.
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
st "bench"; timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"; chk $?
V="$L/librtamd.so $L/variants/librtamd_bytes.so $L/variants/librtamd_nomargin.so"
st "ab c3"; REPS=3 bash tools/ab_lib.sh "$OUT/ab3" "--steps 200 --warmup 5" $V; chk $?
st "ab c5"; REPS=2 bash tools/ab_lib.sh "$OUT/ab5" "--config 5 --steps 20 --warmup 3" $V; chk $?
st done
