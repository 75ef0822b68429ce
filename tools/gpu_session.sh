#!/bin/bash
# One GPU session on the gpurun box: parity tests, smoke, bench, rocprof.
# Each GPU step has its own time limit; a fault / abort / timeout ends the
# session (no further GPU step runs).  Usage: tools/gpu_session.sh TAG [steps...]
# steps: test smoke bench prof pmc ab   (default: test smoke bench prof)
# ab: tools/ab_bench.py with the arguments in $AB_ARGS
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r01}; shift || true
STEPS=${*:-test smoke bench prof}
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
rocminfo 2>/dev/null | grep -m1 -E "gfx950" > "$OUT/rocminfo.txt"
for s in $STEPS; do
  case $s in
    test)  run pytest 900 python -u -m pytest tests -m gpu -q -rA --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
               python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/prof.log" 2>&1 ;;
    pmc)   run pmc 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "trace_(simple|persistent|coop)" --output-format csv \
               -d "$OUT/pmc" -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/pmc.log" 2>&1 ;;
    ab)    run ab 900 python tools/ab_bench.py ${AB_ARGS:-} > "$OUT/ab.jsonl" 2> "$OUT/ab.err" ;;
  esac
done
status "session done"
