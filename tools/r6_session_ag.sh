#!/bin/bash
# Round 6: 4 frames per launch against 2 at the driver's 20 steps (config 3)
# and 10 steps of config 5, four rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
chk() { local rc=$1; st "rc=$rc"; if [ "$rc" -ne 0 ]; then st "abort"; exit "$rc"; fi; }
st "c3"; ARMS_FILE=tools/arms/r6_b20.txt REPS=4 STEPS=20 bash tools/ab_args.sh "$TAG/b3"; chk $?
printf -- '--config 5 --no-pcie --no-lanes\n--config 5 --no-pcie --no-lanes --batch 4\n' > "$OUT/arms5.txt"
st "c5"; ARMS_FILE="$OUT/arms5.txt" REPS=3 STEPS=20 bash tools/ab_args.sh "$TAG/b5"; chk $?
st done
