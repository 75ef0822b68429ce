#!/bin/bash
# Round 6: the forced-record rule (accel_build.h kAccelForce) in place of
# per-record margin factors.  The whole GPU suite and smoke, then A/Bs on one
# box: the build against the per-record factors (classr, the previous tree),
# against round 5's fixed factor (nomargin) and against the compiler's default
# schedule (defsched), configs 3 and 5; then config 3's spans emulation at
# N = 4 with 1 and 2 frames per launch group.
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
st "ab classr c3"; REPS=3 bash tools/ab_lib.sh "$OUT/ab_classr3" "--steps 200 --warmup 5" $L/librtamd.so $L/variants/librtamd_classr.so; chk $?
st "ab nomargin c3"; REPS=3 bash tools/ab_lib.sh "$OUT/ab_nomargin3" "--steps 200 --warmup 5" $L/librtamd.so $L/variants/librtamd_nomargin.so; chk $?
st "ab classr c5"; REPS=2 bash tools/ab_lib.sh "$OUT/ab_classr5" "--config 5 --steps 20 --warmup 3" $L/librtamd.so $L/variants/librtamd_classr.so; chk $?
st "ab nomargin c5"; REPS=2 bash tools/ab_lib.sh "$OUT/ab_nomargin5" "--config 5 --steps 20 --warmup 3" $L/librtamd.so $L/variants/librtamd_nomargin.so; chk $?
st "ab sched c3"; REPS=3 bash tools/ab_lib.sh "$OUT/absched3" "--steps 200 --warmup 5" $L/librtamd.so $L/variants/librtamd_defsched.so; chk $?
st "ab sched c5"; REPS=2 bash tools/ab_lib.sh "$OUT/absched5" "--config 5 --steps 20 --warmup 3" $L/librtamd.so $L/variants/librtamd_defsched.so; chk $?
B="--no-cpu-baseline --no-pcie --no-lanes"
st "n1 c3"; timeout -k 10 300 python bench.py --steps 20 --warmup 5 $B > "$OUT/n1_c3.json" 2> "$OUT/n1_c3.err"; chk $?
for lf in 1 2; do
  st "emu c3 n4 lf$lf"; bash tools/emulate.sh "$OUT/emu" c3lf$lf 4 "0 1" --steps 20 --warmup 5 --span-launch-frames $lf; chk $?
done
st done
