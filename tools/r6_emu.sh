#!/bin/bash
# Round 6 (verdict r05 next #5): the N > 1 paths on the shipped kernel
# (accel 8), rank by rank on one GPU (tools/emulate.sh; BENCH_EMULATE):
#   * config 5 (1M triangles, 4K, 8 bounces) at N = 8, spans (the default):
#     ranks 0, 1, 7;
#   * config 4 (50k, 1080p, 8 bounces) as BASELINE names it: 2 x 2 tiles over
#     N = 4 with the float radiance gathered beside RGBA8: ranks 0-3;
#   * config 3 at N = 8: a rocprofv3 kernel trace of sender rank 1 and of
#     N = 1 in the same session (the sender slowdown).
# N = 1 of each config on the same box first.  Each GPU step under its own
# time limit; a fault, abort or timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "$(date +%T) $*" >> "$OUT/status.txt"; }
chk() { local rc=$1; st "rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then st "abort"; exit "$rc"; fi; }
B="--no-cpu-baseline --no-pcie --no-lanes"
st "n1 cfg3"; timeout -k 10 300 python bench.py --steps 20 --warmup 5 $B > "$OUT/n1_c3.json" 2> "$OUT/n1_c3.err"; chk $?
st "n1 cfg5"; timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 3 $B > "$OUT/n1_c5.json" 2> "$OUT/n1_c5.err"; chk $?
st "n1 cfg4"; timeout -k 10 300 python bench.py --config 4 --steps 20 --warmup 5 $B > "$OUT/n1_c4.json" 2> "$OUT/n1_c4.err"; chk $?
st "emu cfg5 n8"; bash tools/emulate.sh "$OUT/emu" c5 8 "0 1 7" --config 5 --steps 10 --warmup 3; chk $?
st "emu cfg4 tiles n4"; bash tools/emulate.sh "$OUT/emu" c4t 4 "0 1 2 3" --config 4 --partition tiles --gather radiance \
    --steps 20 --warmup 5; chk $?
# the sender slowdown: kernel traces of N = 1 and of an emulated N = 8 sender
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1
st "trace n1"
MASTER_PORT=29611 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr_n1" -o run -- \
    python3 bench.py --steps 20 --warmup 5 $B > "$OUT/tr_n1.json" 2> "$OUT/tr_n1.err"; chk $?
st "trace n8 r1"
BENCH_EMULATE=8:1 MASTER_PORT=29612 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/tr_n8r1" -o run -- python3 bench.py --steps 20 --warmup 5 $B --no-single > "$OUT/tr_n8r1.json" \
    2> "$OUT/tr_n8r1.err"; chk $?
st "trace n8 r0"
BENCH_EMULATE=8:0 MASTER_PORT=29613 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/tr_n8r0" -o run -- python3 bench.py --steps 20 --warmup 5 $B --no-single > "$OUT/tr_n8r0.json" \
    2> "$OUT/tr_n8r0.err"; chk $?
st done
