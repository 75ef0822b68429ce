#!/bin/bash
# Round 6: span launch groups (--span-launch-frames): their GPU parity tests,
# then the N > 1 emulation (tools/emulate.sh, one rank alone on the GPU) of
# config 3 at N = 8 and N = 2 with 1, 2 and 3 frames per launch group, and of
# config 5 at N = 8 with 1 and 2, against N = 1 on the same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
chk() { local rc=$1; st "rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then st "abort"; exit "$rc"; fi; }
st "pytest"; timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_parity.py -m gpu -q -rA \
    --timeout 300 --timeout-method thread -k "span or runs or rect or tile_exchange" > "$OUT/pytest.log" 2>&1; chk $?
B="--no-cpu-baseline --no-pcie --no-lanes"
for rep in 1 2; do
  st "n1 c3 $rep"; timeout -k 10 300 python bench.py --steps 20 --warmup 5 $B > "$OUT/n1_c3_$rep.json" 2> "$OUT/n1_c3_$rep.err"; chk $?
  for lf in 1 2 3; do
    st "emu c3 n8 lf$lf $rep"; bash tools/emulate.sh "$OUT/emu" c3lf${lf}_$rep 8 "0 1" --steps 20 --warmup 5 \
        --span-launch-frames $lf; chk $?
    st "emu c3 n2 lf$lf $rep"; bash tools/emulate.sh "$OUT/emu" c3lf${lf}_$rep 2 "0 1" --steps 20 --warmup 5 \
        --span-launch-frames $lf; chk $?
  done
done
st "n1 c5"; timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 3 $B > "$OUT/n1_c5.json" 2> "$OUT/n1_c5.err"; chk $?
for lf in 1 2; do
  st "emu c5 n8 lf$lf"; bash tools/emulate.sh "$OUT/emu" c5lf$lf 8 "0 1" --config 5 --steps 10 --warmup 3 \
      --span-launch-frames $lf; chk $?
done
st done
