#!/bin/bash
# PMC passes A and D plus per-wave timelines for walk 0 and walk 1 (profiles/r01/walks.md).
set -o pipefail
RTAMD_WALK=0 PMC_PASSES="A D" bash tools/pmc.sh ${TAG:-r01s}_w0 && RTAMD_WALK=1 PMC_PASSES="A D" bash tools/pmc.sh ${TAG:-r01s}_w1 && \
for w in 0 1; do for b in 1 4; do RTAMD_WALK=$w timeout -k 10 300 python tools/diag_timeline.py --wave-tile 2 --bounces $b --out gpurun_out/${TAG:-r01s}_diag_w${w}b${b}.npz > gpurun_out/${TAG:-r01s}_diag_w${w}b${b}.txt 2>&1 || exit 3; done; done
