#!/bin/bash
# Round 6: option accel_octants (fewer of the 8 layouts walked):
# its GPU tests, then bench arms on configs 3 and 5 (masks 5, 3, 6)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
chk() { local rc=$1; st "rc=$rc"; if [ "$rc" -ne 0 ]; then st "abort"; exit "$rc"; fi; }
st "pytest"; timeout -k 10 600 python -u -m pytest tests/test_gpu_accel.py -m gpu -q -rA --timeout 300 \
    --timeout-method thread -k "octants" > "$OUT/pytest.log" 2>&1; chk $?
st "c3"; ARMS_FILE=tools/arms/r6_oct3.txt REPS=3 STEPS=200 bash tools/ab_args.sh "$TAG/oct3"; chk $?
st "c5"; ARMS_FILE=tools/arms/r6_oct5.txt REPS=2 STEPS=20 bash tools/ab_args.sh "$TAG/oct5"; chk $?
st done
