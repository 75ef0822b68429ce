#!/bin/bash
# Session r2k1 (one GPU): the RCCL exchange path (GPU test at world size 1,
# bench.py's N > 1 code path forced at world size 1 over RCCL, and two ranks
# sharing the GPU over RCCL if RCCL allows it), then an A/B of non-temporal
# frame stores (build flag RT_NT_STORE, library in build_nt/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2k1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
fatal() { local rc=$1; [ $rc -ne 0 ] && [ $rc -ne 1 ] && { st "abort rc=$rc"; exit $rc; }; return 0; }
port() { echo $((29500 + RANDOM % 1000)); }

st "start pytest_dist"
timeout -k 10 180 python -u -m pytest tests/test_gpu_dist.py -m gpu -v --timeout 120 --timeout-method thread \
  > "$OUT/pytest_dist.log" 2>&1; rc=$?; st "end pytest_dist rc=$rc"; fatal $rc

st "start forced_dist_n1"
BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port $(port) bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
  > "$OUT/bench_forced_dist_nccl_n1.json" 2> "$OUT/bench_forced_dist_nccl_n1.err"; rc=$?
st "end forced_dist_n1 rc=$rc"; fatal $rc

st "start share_nccl_n2"
BENCH_SHARE_GPU=1 BENCH_DIST_BACKEND=nccl timeout -k 10 180 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $(port) bench.py --gpus 2 --steps 20 --warmup 5 \
  --no-cpu-baseline > "$OUT/bench_bands_nccl_n2_shared.json" 2> "$OUT/bench_bands_nccl_n2_shared.err"; rc=$?
st "end share_nccl_n2 rc=$rc"; fatal $rc

NT=3d-ray-tracer-vulkan_amd/build_nt/lib/librtamd.so
for rep in 1 2 3; do
  for arm in base nt; do
    lp=""; [ $arm = nt ] && lp=$NT
    st "start c3 $arm $rep"
    RTAMD_LIB_PATH=$lp timeout -k 10 300 python bench.py --steps 200 --warmup 5 --no-cpu-baseline \
      > "$OUT/c3_${arm}_$rep.json" 2>> "$OUT/ab.err"; rc=$?; st "end rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
for rep in 1 2; do
  for arm in base nt; do
    lp=""; [ $arm = nt ] && lp=$NT
    st "start c5 $arm $rep"
    RTAMD_LIB_PATH=$lp timeout -k 10 300 python bench.py --config 5 --steps 20 --warmup 3 --no-cpu-baseline \
      > "$OUT/c5_${arm}_$rep.json" 2>> "$OUT/ab.err"; rc=$?; st "end rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
st "session done"
