#!/bin/bash
# Walk 13 (top tree in LDS): its parity tests first, then bench A/B against
# the default (200 steps, alternated).  Every GPU step has its own limit; a
# failure ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export GPU_MAX_HW_QUEUES=16
TAG=${1:-r2top}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() { local name=$1 secs=$2; shift 2; echo "$(date +%T) start $name" >> "$OUT/status.txt"
  timeout -k 10 "$secs" "$@"; local rc=$?; echo "$(date +%T) end $name rc=$rc" >> "$OUT/status.txt"; return $rc; }
step pytest_top 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rA --timeout 120 --timeout-method thread \
    -k "top_tree or schedules_identical or unbalanced or spheres_bit_exact" > "$OUT/pytest_top.log" 2>&1 || exit $?
for r in ${AB_REPS:-1 2}; do
  for arm in ${ARMS:-base w13 w13b8}; do
    lib_=""; lv_=64
    case $arm in
      base) set_="" ;;
      w13) set_="walk=13" ;;
      w13b8) set_="walk=13,block_waves=8" ;;
      w13t11) set_="walk=13"; lib_=$PWD/build_top11/librtamd.so ;;   # 11-bit slots: 2047 top nodes, 64 KB LDS
      w13L0) set_="walk=13"; lv_=0 ;;                                  # empty top tree: the workgroup shape alone
      w13b8L0) set_="walk=13,block_waves=8"; lv_=0 ;;
      *) set_="${arm//:/=}" ;;
    esac
    for c in ${CFGS:-3}; do
      n=200; [ "$c" = 5 ] && n=20
      RTAMD_TOP_LEVELS=$lv_ RTAMD_LIB_PATH=$lib_ step ${arm}_c${c}_$r 180 python bench.py --config $c --steps $n --warmup 5 --no-cpu-baseline ${set_:+--set $set_} \
          > "$OUT/ab_${arm}_c${c}_$r.json" 2> "$OUT/ab_${arm}_c${c}_$r.err" || exit $?
    done
  done
done
echo "$(date +%T) session done" >> "$OUT/status.txt"
