#!/bin/bash
# Session r2k13 (one GPU): non-temporal leaf-record loads (build flag
# RT_NT_LEAF, library in build_ntl/) vs the default, configs 5 and 3, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2k13}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
NTL=3d-ray-tracer-vulkan_amd/build_ntl/lib/librtamd.so
ab() { local tag=$1 lp=$2; shift 2; st "start $tag"; RTAMD_LIB_PATH=$lp timeout -k 10 300 python bench.py \
  --no-cpu-baseline "$@" > "$OUT/$tag.json" 2>> "$OUT/ab.err"; local rc=$?; st "end rc=$rc"; return $rc; }
for rep in 1 2 3; do
  ab c5_base_$rep "" --config 5 --steps 20 --warmup 3 || exit $?
  ab c5_ntl_$rep $NTL --config 5 --steps 20 --warmup 3 || exit $?
done
for rep in 1 2; do
  ab c3_base_$rep "" --steps 200 || exit $?
  ab c3_ntl_$rep $NTL --steps 200 || exit $?
done
st "session done"
