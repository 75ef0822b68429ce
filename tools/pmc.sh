#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 process per counter set;
# --pmc is never combined with other tracing).  Usage: tools/pmc.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
pass() {  # pass NAME COUNTERS...
  local name=$1; shift
  echo "$(date +%T) pass $name: $*" >> "$OUT/status.txt"
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex "trace_(simple|persistent|coop)" --output-format csv \
      -d "$OUT/$name" -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-pcie --no-lanes ${BENCH_ARGS:-} > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$(date +%T) pass $name rc=$rc" >> "$OUT/status.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
PASSES=${PMC_PASSES:-"A B C D E"}
for p in $PASSES; do
  case $p in
    A) pass A SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU ;;
    B) pass B TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum ;;
    C) pass C FETCH_SIZE ;;
    D) pass D SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE TA_BUSY_avr ;;
    E) pass E TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_REQ_sum ;;
    F) pass F SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_LEVEL_WAVES SQ_INSTS_SMEM SQ_BUSY_CU_CYCLES ;;
    G) pass G TCP_TCP_LATENCY_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum ;;
    H) pass H TCP_TOTAL_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_TA_BUSY_sum TA_TOTAL_WAVEFRONTS_sum SQ_INSTS_BRANCH SQ_INST_LEVEL_SMEM ;;
  esac
done
echo "$(date +%T) pmc done" >> "$OUT/status.txt"
