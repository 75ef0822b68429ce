#!/bin/bash
# Round 6: rank 0's span weight on the final tree (spans, two frames per launch
# group), emulated: N = 2 at 1.0 (default) and 1.1, N = 4 at 0.9 (default) and
# 1.0; 20 steps, two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
chk() { local rc=$1; st "rc=$rc"; if [ "$rc" -ne 0 ]; then st "abort"; exit "$rc"; fi; }
for rep in 1 2; do
  for w in 1.0 1.1; do
    st "n2 w$w $rep"; bash tools/emulate.sh "$OUT/emu" n2w${w}_$rep 2 "0 1" --steps 20 --warmup 5 --root-weight $w; chk $?
  done
  for w in 0.9 1.0; do
    st "n4 w$w $rep"; bash tools/emulate.sh "$OUT/emu" n4w${w}_$rep 4 "0 1" --steps 20 --warmup 5 --root-weight $w; chk $?
  done
done
st done
