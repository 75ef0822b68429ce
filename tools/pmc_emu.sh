#!/bin/bash
# PMC passes (tools/pmc.sh's A and B) of one rank of an N-rank bench.py run
# emulated on this GPU (BENCH_EMULATE=N:r, no exchange: BENCH_EMULATE_NOX=1),
# without a launcher: the rendezvous variables are exported here, so the
# program after rocprofv3's "--" is python3 itself.
# Usage: tools/pmc_emu.sh OUTDIR N RANK [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$1; N=$2; R=$3; shift 3
mkdir -p "$OUT"
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29500 + RANDOM % 1000))
export BENCH_EMULATE=$N:$R BENCH_EMULATE_NOX=1
for p in A B; do
  case $p in
    A) C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" ;;
    B) C="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" ;;
  esac
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "trace_simple" --output-format csv \
      -d "$OUT/$p" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --no-single "$@" \
      > "$OUT/$p.log" 2>&1 || exit $?
done
