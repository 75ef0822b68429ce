#!/bin/bash
# Round 6: PMC passes A (instruction counts) and D (waits, LDS, TA) of the
# default binary walk and of option accel_wide on config 3 and 5, then
# config 5 with one accel layout (accel 1) against 8, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
for c in 3 5; do
  PMC_PASSES="A D" BENCH_ARGS="--config $c" bash tools/pmc.sh "${TAG}_b8_c$c" || exit $?
  RTAMD_ACCEL_WIDE=1 PMC_PASSES="A D" BENCH_ARGS="--config $c" bash tools/pmc.sh "${TAG}_wide_c$c" || exit $?
done
for i in 1 2; do
  for nl in 8 1; do
    st "start cfg5 accel $nl $i"
    RTAMD_ACCEL=$nl timeout -k 10 300 python bench.py --config 5 --steps 20 --warmup 3 --no-cpu-baseline --no-pcie \
        > "$OUT/c5_a${nl}_$i.json" 2> "$OUT/c5_a${nl}_$i.err"
    rc=$?; st "rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
done
st done
