# r3v2: the frame kernel built with LLVM's AMDGPU scheduler strategies
# (build_v/<variant>/librtamd.so, loaded through RTAMD_LIB_PATH) against the
# default build, interleaved three times at 200 steps, then config 5 once.
set -u
O=gpurun_out/r3v2b
mkdir -p $O
run() {  # run VARIANT TAG ARGS...
  local v=$1 tag=$2; shift 2
  local L=""
  [ "$v" != def ] && L=build_v/$v/librtamd.so
  RTAMD_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie "$@" > $O/$tag.json 2> $O/$tag.err || exit $?
}
for rep in a b c; do
  for v in def mclause ilp bias; do run $v ${v}_$rep --steps 200; done
done
for v in def mclause ilp; do run $v c5_$v --config 5 --steps 10 --warmup 3; done
echo done > $O/done.txt
