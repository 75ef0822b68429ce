# r3v3: the max-ILP build as the tree's library: every GPU parity test, then
# A/B against the default-strategy build (build_v/def) interleaved three times
# at 200 and at 20 steps, configs 5 and 6 once.
set -u
O=gpurun_out/r3v3
mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> $O/pytest_gpu.log
run() {  # run VARIANT TAG ARGS...
  local v=$1 tag=$2; shift 2
  local L=""
  [ "$v" != new ] && L=build_v/$v/librtamd.so
  RTAMD_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie "$@" > $O/$tag.json 2> $O/$tag.err || exit $?
}
for rep in a b c; do
  for v in def new; do run $v ${v}200_$rep --steps 200; run $v ${v}20_$rep --steps 20; done
done
for v in def new; do run $v c5_$v --config 5 --steps 10 --warmup 3; run $v c6_$v --config 6 --steps 100; done
echo done > $O/done.txt
