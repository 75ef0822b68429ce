#!/bin/bash
# Session r2k16 (one GPU): re-sweep of heavy_pixel_factor and coop_lanes on
# the final round-2 default (config 3, 200 steps; config 6 for the factor),
# two interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2k16}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
ab() { local tag=$1; shift; st "start $tag"; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" \
  > "$OUT/$tag.json" 2>> "$OUT/ab.err"; local rc=$?; st "end rc=$rc"; return $rc; }
for rep in 1 2; do
  for hpf in 35 50 65; do ab c3_hpf${hpf}_$rep --steps 200 --set heavy_pixel_factor=$hpf || exit $?; done
  ab c3_coop2_$rep --steps 200 --set coop_lanes=2 || exit $?
  for hpf in 35 50 65; do ab c6_hpf${hpf}_$rep --config 6 --steps 200 --set heavy_pixel_factor=$hpf || exit $?; done
done
st "session done"
