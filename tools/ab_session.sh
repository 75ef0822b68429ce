#!/bin/bash
# A/B on one GPU box: parity tests, then bench.py variants (3 runs each, 200
# steps), then the N>1 rehearsal (ranks sharing the GPU, gloo).
# Variants: "ENV=VAL ... -- bench args" lines in $AB_FILE (default: graph 0/1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
i=0
while IFS= read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1)); envs=${line%%--*}; bargs=${line#*--}
  for r in 1 2 3; do
    env $envs timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu-baseline $bargs > $O/v${i}_$r.json 2> $O/v${i}_$r.err || exit 1
    echo "v$i r$r [$line] $(tail -n 1 $O/v${i}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"], d["config"]["schedule"])')" >> $O/summary.txt
  done
done < "${AB_FILE:-/dev/null}"
if [ -n "${DIST:-}" ]; then
  for n in $DIST; do TAG=${TAG:-ab}_dist NPROC=$n BACKENDS=gloo bash tools/dist_rehearsal.sh || exit 1; done
fi
