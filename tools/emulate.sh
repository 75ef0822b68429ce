#!/bin/bash
# bench.py's N > 1 bands partition, one rank at a time on one GPU
# (BENCH_EMULATE=N:r; analysis only).  Usage:
#   tools/emulate.sh OUTDIR TAG N "RANKS" [bench args...]
# writes OUTDIR/TAG_nN_rR.json per rank.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; TAG=$2; N=$3; RANKS=$4; shift 4
mkdir -p "$OUT"
for r in $RANKS; do
  BENCH_EMULATE=$N:$r timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --no-cpu-baseline --no-pcie --no-single "$@" \
    > "$OUT/${TAG}_n${N}_r${r}.json" 2> "$OUT/${TAG}_n${N}_r${r}.err" || exit $?
done
