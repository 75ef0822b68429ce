#!/bin/bash
# A/B of bench.py arms that differ by environment (e.g. RTAMD_ACCEL=1),
# interleaved round by round on one GPU box.  Usage:
#   tools/ab_env.sh OUTDIR REPS "ARM_ENV_1" "ARM_ENV_2" ... -- BENCH_ARGS...
# An arm is a space-separated list of NAME=VALUE (or "-" for none).  Each run
# writes OUTDIR/armK_repR.json; a summary line per run goes to OUTDIR/ab.txt.
set -u
out=$1; reps=$2; shift 2
arms=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do arms+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
mkdir -p "$out"
for r in $(seq 1 "$reps"); do
  for k in "${!arms[@]}"; do
    a=${arms[$k]}
    [ "$a" = "-" ] && a=""
    f="$out/arm${k}_rep${r}.json"
    timeout -k 10 300 env $a python3 bench.py --no-cpu-baseline --no-pcie --no-lanes "$@" > "$f" 2> "$out/arm${k}_rep${r}.err"
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "arm $k rep $r rc=$rc: stop" >> "$out/ab.txt"; exit $rc; fi
    python3 - "$f" "$k" "$r" "$a" >> "$out/ab.txt" <<'EOF'
import json, sys
f, k, r, a = sys.argv[1:]
try:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f"arm {k} rep {r} [{a}] ms_per_step {d['ms_per_step']:.4f} value {d['value']:.1f} "
          f"verified {d['config'].get('frames_verified')}")
except Exception as e:
    print(f"arm {k} rep {r} [{a}] no result ({e})")
EOF
  done
done
