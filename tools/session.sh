#!/bin/bash
# One GPU session on a gpurun box (replaces round 2's per-session scripts).
# Every GPU step runs under its own time limit; a fault, abort or timeout
# (exit status other than 0 / 1) ends the session, so nothing else touches the
# GPU after it.  Usage: tools/session.sh TAG step [step ...]
#
#   test      pytest -m gpu (every GPU parity test)
#   smoke     __graft_entry__.smoke()
#   bench     bench.py at the driver's 20 steps / 5 warmup (config 3)
#   bench200  bench.py with its default 200 steps
#   prof3     rocprofv3 --kernel-trace --stats of bench.py --steps 20, then
#             tools/rocprof_union.py (device union per frame vs ms_per_step)
#   prof5     the same for config 5 (--steps 10)
#   pmc3      PMC passes A (SQ instruction counts) and C (FETCH_SIZE) of
#             config 3, merged into gpurun_out/TAG/pmc_latest.json
#   pmc5      the same for config 5
#   fetch5    pmc5 with coop_lanes 0 (no cooperative tail) and with order_split 40
#   pmc3o     the same for config 3 with the orbiting camera (record key cfg3_...@orbit)
#   orbit     bench.py --camera-path orbit at 20 steps
#   cfgs      bench.py on configs 4, 5, 6
#   inflight  bench.py at 1, 2 and 4 ($INFLIGHT) launches in flight (200 steps): the headline
#             frac must not move with them
#   share     tools/share_inflight_bench.py (one rank's share, frames in flight)
#   emu       tools/rank_emulator.py (one rank of N with its exchange; $EMU_ARGS)
#   pipeline  tools/pipeline_bench.py (PCIe-inclusive rates)
#   spawn2    bench.py --gpus 2 with no launcher (it starts its own ranks):
#             BENCH_SHARE_GPU=1 BENCH_DIST_BACKEND=gloo, two gloo ranks on one GPU
#   spawn4    the same with 4 ranks and the 2 x 2 tile grid + radiance gather
#   ab3 / ab5 bench.py interleaved against the tree in build_ab/old (tools/ab_old_new.sh),
#             config 3 (3 rounds, 200 steps) / config 5 (2 rounds, 10 steps)
#   abargs    tools/ab_args.sh over the arms in $ARMS_FILE ($REPS rounds, $STEPS steps)
#   cmd       the command in $CMD (600 s)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
status() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
run() {  # run NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  status "start $name"
  timeout -k 10 "$secs" "$@"
  local rc=$?
  status "end $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then status "abort session (rc=$rc)"; exit $rc; fi
  return 0
}
prof() {  # prof CONFIG STEPS
  local c=$1 k=$2 d="$OUT/prof$1"
  run "prof$c" 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- \
      python3 bench.py --config "$c" --steps "$k" --warmup 5 --no-cpu-baseline --no-pcie > "$OUT/prof$c.json" 2> "$OUT/prof$c.err"
  local tr
  tr=$(find "$d" -name "run_kernel_trace.csv" | head -n 1)
  python3 tools/rocprof_union.py "$tr" --steps "$k" --bench "$OUT/prof$c.json" --out "$OUT/union_cfg$c.json" \
      > /dev/null 2>> "$OUT/status.txt" || status "rocprof_union cfg$c failed"
  cp "$(find "$d" -name "run_kernel_stats.csv" | head -n 1)" "$OUT/kernel_stats_cfg$c.csv" 2>/dev/null || true
}
pmc() {  # pmc CONFIG NAME [SUFFIX EXTRA_BENCH_ARGS]
  local c=$1 name=$2 sfx=${3:-} extra=${4:-}
  PMC_PASSES="A C" BENCH_ARGS="--config $c $extra" bash tools/pmc.sh "${TAG}_pmc$c$sfx" || exit $?
  cp -r "gpurun_out/${TAG}_pmc$c$sfx" "$OUT/pmc$c$sfx"
  python3 tools/pmc_traffic.py "gpurun_out/${TAG}_pmc$c$sfx" "trace_simple<false, false" --config "$name" \
      --source "profiles/r06/$TAG/pmc$c$sfx (tools/pmc.sh passes A and C, bench.py --config $c $extra)" \
      --merge "$OUT/pmc_latest.json" > "$OUT/pmc$c$sfx.json" 2>> "$OUT/status.txt" || status "pmc_traffic cfg$c$sfx failed"
  cp "$OUT/pmc_latest.json" profiles/pmc_latest.json
}
rocminfo 2>/dev/null | grep -m1 -E "gfx950" > "$OUT/rocminfo.txt"
# PMC records accumulate onto the committed ones; after a pmc step the box's
# profiles/pmc_latest.json is the merged file, so later bench steps of the
# session attach the fresh records (copy gpurun_out/TAG/pmc_latest.json back)
[ -f "$OUT/pmc_latest.json" ] || cp profiles/pmc_latest.json "$OUT/pmc_latest.json"
for s in "$@"; do
  case $s in
    test)     run pytest 1200 python -u -m pytest tests -m gpu -q -rA --timeout 120 --timeout-method thread \
                  > "$OUT/pytest_gpu.log" 2>&1 ;;
    smoke)    run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    bench)    run bench 600 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    bench200) run bench200 600 python bench.py > "$OUT/bench200.json" 2> "$OUT/bench200.err" ;;
    prof3)    prof 3 20 ;;
    prof5)    prof 5 10 ;;
    # record keys: bench.py pmc_key (the default accel 8 walk: "@accel8"; the N = 1 default of 4 frames per launch: "@f4")
    pmc3)     pmc 3 cfg3_50k_1920x1080_b4@accel8@f4 ;;
    pmc5)     pmc 5 cfg5_1M_3840x2160_b8@accel8@f4 ;;
    pmc6)     pmc 6 cfg6_fbm_1920x1080_b4@accel8@f4 ;;
    pmc3r)    RTAMD_ACCEL=0 pmc 3 cfg3_50k_1920x1080_b4 r ;;
    fetch5)   pmc 5 cfg5_1M_3840x2160_b8@nocoop@accel8@f4 n "--set coop_lanes=0" && \
              pmc 5 cfg5_1M_3840x2160_b8@split40@accel8@f4 s "--set order_split=40" ;;
    pmc3o)    pmc 3 cfg3_50k_1920x1080_b4@orbit@accel8 o "--camera-path orbit --batch 1" ;;
    orbit)    run orbit 600 python bench.py --steps 20 --warmup 5 --camera-path orbit \
                  > "$OUT/bench_orbit.json" 2> "$OUT/bench_orbit.err" ;;
    cfgs)     for a in "4 50" "5 10" "6 200"; do
                set -- $a
                run "cfg$1" 300 python bench.py --config "$1" --steps "$2" --warmup 3 --no-cpu-baseline \
                    > "$OUT/bench_cfg$1.json" 2> "$OUT/bench_cfg$1.err"
              done ;;
    inflight) for k in ${INFLIGHT:-1 2 4}; do
                run "inflight$k" 300 python bench.py --inflight "$k" --steps 200 --warmup 5 --no-cpu-baseline \
                    --no-pcie > "$OUT/bench_if$k.json" 2> "$OUT/bench_if$k.err"
              done ;;
    share)    run share 600 python tools/share_inflight_bench.py ${SHARE_ARGS:-} > "$OUT/share.jsonl" 2> "$OUT/share.err" ;;
    emu)      run emu 900 python tools/rank_emulator.py ${EMU_ARGS:-} > "$OUT/emu.jsonl" 2> "$OUT/emu.err" ;;
    pipeline) run pipeline 300 python tools/pipeline_bench.py ${PIPE_ARGS:-} > "$OUT/pipeline.jsonl" 2> "$OUT/pipeline.err" ;;
    spawn2)   run spawn2 600 env BENCH_SHARE_GPU=1 BENCH_DIST_BACKEND=gloo python bench.py --gpus 2 --steps 20 \
                  --warmup 5 > "$OUT/spawn2.json" 2> "$OUT/spawn2.err" ;;
    spawn4)   run spawn4 600 env BENCH_SHARE_GPU=1 BENCH_DIST_BACKEND=gloo python bench.py --gpus 4 --steps 10 \
                  --warmup 3 --partition tiles --gather radiance > "$OUT/spawn4.json" 2> "$OUT/spawn4.err" ;;
    ab3)      run ab3 900 bash tools/ab_old_new.sh "$OUT/ab3" 3 --steps 200 --warmup 5 ;;
    ab5)      run ab5 900 bash tools/ab_old_new.sh "$OUT/ab5" 2 --config 5 --steps 10 --warmup 3 ;;
    abargs)   run abargs 900 env ARMS_FILE="${ARMS_FILE:?}" REPS="${REPS:-3}" STEPS="${STEPS:-200}" \
                  bash tools/ab_args.sh "$TAG/abargs_$(basename "$ARMS_FILE" .txt)" ;;
    cmd)      run cmd 600 bash -c "$CMD" > "$OUT/cmd.log" 2>&1 ;;
    *)        status "unknown step $s" ;;
  esac
done
status "session done"
