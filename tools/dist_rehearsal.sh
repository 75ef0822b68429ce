#!/bin/bash
# Rehearse bench.py's N>1 paths on a 1-GPU box: NPROC ranks share the GPU
# (BENCH_SHARE_GPU=1; the JSON says so).  The real 1/2/4/8-GPU runs are the
# driver's.  Every artifact carries bench.py's sha (bench_sha16).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-dist}
mkdir -p "$OUT"
for part in ${PARTS:-bands frames}; do
  for be in ${BACKENDS:-nccl gloo}; do
    BENCH_SHARE_GPU=1 BENCH_DIST_BACKEND=$be timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node ${NPROC:-2} --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus ${NPROC:-2} \
      --steps ${STEPS:-24} --warmup 3 --partition $part > "$OUT/bench_${part}_${be}_n${NPROC:-2}.json" 2> "$OUT/bench_${part}_${be}_n${NPROC:-2}.err"
    rc=$?
    echo "$part $be n=${NPROC:-2} rc=$rc" >> "$OUT/status.txt"
    if [ $rc -eq 0 ]; then break; fi
    if [ $rc -ne 1 ]; then exit $rc; fi
  done
done
