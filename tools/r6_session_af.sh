#!/bin/bash
# Round 6: the final tree's launch knobs: frames per launch (2, 4) and
# launches in flight (4, 3, 6), configs 3 and 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
chk() { local rc=$1; st "rc=$rc"; if [ "$rc" -ne 0 ]; then st "abort"; exit "$rc"; fi; }
st "c3"; ARMS_FILE=tools/arms/r6_final3.txt REPS=3 STEPS=200 bash tools/ab_args.sh "$TAG/k3"; chk $?
st "c5"; ARMS_FILE=tools/arms/r6_final5.txt REPS=2 STEPS=20 bash tools/ab_args.sh "$TAG/k5"; chk $?
st done
