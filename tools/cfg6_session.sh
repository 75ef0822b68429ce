#!/bin/bash
# Config 6 (the reference's FinalBaseMesh): GPU parity suite, bench line and
# rocprofv3 kernel stats.  Every GPU step has its own limit; a failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-cfg6}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -rA --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config 6 --steps 20 --warmup 5 > $O/bench_cfg6.json 2> $O/bench_cfg6.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --config 6 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
python tools/rocprof_frames.py $O/prof/run_kernel_trace.csv > $O/rocprof_frames.json
