#!/bin/bash
# Round 6: frames per launch 4, 5 and 10 at the
# driver's 20 steps, config 3, four rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
chk() { local rc=$1; st "rc=$rc"; if [ "$rc" -ne 0 ]; then st "abort"; exit "$rc"; fi; }
st "c3"; ARMS_FILE=tools/arms/r6_b5.txt REPS=4 STEPS=20 bash tools/ab_args.sh "$TAG/i3"; chk $?
st done
