set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for i in 1 2 3; do
  RTAMD_GRAPH=0 timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > $O/g0_$i.json 2> $O/g0_$i.err || exit 1
  RTAMD_GRAPH=1 timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > $O/g1_$i.json 2> $O/g1_$i.err || exit 1
done
