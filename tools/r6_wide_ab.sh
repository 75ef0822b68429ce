#!/bin/bash
# Round 6: option accel_wide (the 4-wide tree) on the GPU: its parity tests,
# then bench.py A/B against the default 8-layout binary walk, interleaved
# (config 3 at 200 steps, config 5 at 20), REPS rounds.  Each GPU step under
# its own time limit; a fault, abort or timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}; REPS=${2:-2}; TESTS=${3:-1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
chk() { local rc=$1; st "rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then st "abort"; exit "$rc"; fi; }
if [ "$TESTS" = 1 ]; then
  st "start pytest accel"
  timeout -k 10 900 python -u -m pytest tests/test_gpu_accel.py -q -rA --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
      > "$OUT/pytest_accel.log" 2>&1; chk $?
fi
for i in $(seq 1 "$REPS"); do
  for arm in b8 wide; do
    env=""; [ "$arm" = wide ] && env="RTAMD_ACCEL_WIDE=1"
    st "start cfg3 $arm $i"
    env $env timeout -k 10 300 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-pcie \
        > "$OUT/c3_${arm}_$i.json" 2> "$OUT/c3_${arm}_$i.err"; chk $?
    st "start cfg5 $arm $i"
    env $env timeout -k 10 300 python bench.py --config 5 --steps 20 --warmup 3 --no-cpu-baseline --no-pcie \
        > "$OUT/c5_${arm}_$i.json" 2> "$OUT/c5_${arm}_$i.err"; chk $?
  done
done
st "done"
