#!/bin/bash
# PMC passes A, B, D for two schedules (BENCH_ARGS per arm), one rocprofv3 per pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-pmcab}
i=0
for arm in "${ARM1:---set walk=2,heavy_tiles=0}" "${ARM2:---set walk=3,heavy_tiles=0}"; do
  i=$((i+1))
  BENCH_ARGS="$arm" PMC_PASSES="${PASSES:-A B D}" bash tools/pmc.sh "${TAG}_arm$i" || exit $?
done
