#!/bin/bash
# bench.py's N > 1 paths rehearsed on a 1-GPU box: NPROC gloo ranks share the
# GPU (BENCH_SHARE_GPU=1, BENCH_DIST_BACKEND=gloo; RCCL refuses two ranks on
# one GPU).  Their rates measure ranks contending for one GPU, not scaling;
# what they check is the partition, the exchange and the assembled frames
# (config.frames_verified).  Usage: tools/rehearse.sh OUTDIR NPROC PARTITION [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; NP=$2; PART=$3; shift 3
mkdir -p "$OUT"
BENCH_SHARE_GPU=1 BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node "$NP" --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus "$NP" \
  --partition "$PART" --no-single "$@" > "$OUT/bench_${PART}_n${NP}.json" 2> "$OUT/bench_${PART}_n${NP}.err"
