#!/bin/bash
# Round 6: the whole GPU suite and smoke on this tree; the cost of the
# thin-triangle margins (A/B against a build with round 5's fixed factor,
# RT_THIN_MARGIN=0); config 4 at N = 4 emulated rank by rank as 2 x 2 tiles
# (F frames' tiles per launch) and as spans.  Each GPU step under its own
# time limit; a fault, abort or timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
chk() { local rc=$1; st "rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then st "abort"; exit "$rc"; fi; }
st "pytest"; timeout -k 10 1200 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1; chk $?
st "smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; chk $?
st "bench"; timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"; chk $?
st "ab margin c3"; REPS=3 bash tools/ab_lib.sh "$OUT/ab3" "--steps 200 --warmup 5" \
    3d-ray-tracer-vulkan_amd/lib/librtamd.so 3d-ray-tracer-vulkan_amd/lib/variants/librtamd_nomargin.so; chk $?
st "ab margin c5"; REPS=2 bash tools/ab_lib.sh "$OUT/ab5" "--config 5 --steps 20 --warmup 3" \
    3d-ray-tracer-vulkan_amd/lib/librtamd.so 3d-ray-tracer-vulkan_amd/lib/variants/librtamd_nomargin.so; chk $?
st "n1 cfg4"; timeout -k 10 300 python bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline --no-pcie --no-lanes \
    > "$OUT/n1_c4.json" 2> "$OUT/n1_c4.err"; chk $?
st "emu cfg4 tiles"; bash tools/emulate.sh "$OUT/emu" c4t 4 "0 1 2 3" --config 4 --partition tiles --gather radiance \
    --steps 20 --warmup 5; chk $?
st "emu cfg4 spans"; bash tools/emulate.sh "$OUT/emu" c4s 4 "0 1 3" --config 4 --gather radiance --steps 20 --warmup 5; chk $?
st "ab sched c3"; REPS=3 bash tools/ab_lib.sh "$OUT/absched" "--steps 200 --warmup 5" \
    3d-ray-tracer-vulkan_amd/lib/librtamd.so 3d-ray-tracer-vulkan_amd/lib/variants/librtamd_defsched.so; chk $?
st "knobs c3"; ARMS_FILE=tools/arms/r6_knobs.txt REPS=3 STEPS=200 bash tools/ab_args.sh "$TAG/knobs"; chk $?
st done
