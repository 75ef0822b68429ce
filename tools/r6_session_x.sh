#!/bin/bash
# Round 6: the final tree at N > 1, emulated rank by rank on one GPU
# (tools/emulate.sh, bench.py defaults: spans, two frames per launch group)
# against N = 1 on the same box: config 3 at N = 2, 4, 8 and config 5 at N = 8,
# the driver's 20 steps, two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
chk() { local rc=$1; st "rc=$rc"; if [ "$rc" -ne 0 ]; then st "abort"; exit "$rc"; fi; }
B="--no-cpu-baseline --no-pcie --no-lanes"
for rep in 1 2; do
  st "n1 c3 $rep"; timeout -k 10 300 python bench.py --steps 20 --warmup 5 $B > "$OUT/n1_c3_$rep.json" 2> "$OUT/n1_c3_$rep.err"; chk $?
  for n in 2 4 8; do
    st "emu c3 n$n $rep"; bash tools/emulate.sh "$OUT/emu" c3_$rep $n "0 1" --steps 20 --warmup 5; chk $?
  done
done
st "n1 c5"; timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 3 $B > "$OUT/n1_c5.json" 2> "$OUT/n1_c5.err"; chk $?
st "emu c5 n8"; bash tools/emulate.sh "$OUT/emu" c5 8 "0 1" --config 5 --steps 10 --warmup 3; chk $?
st done
