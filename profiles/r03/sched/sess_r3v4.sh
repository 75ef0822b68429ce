# r3v4: the iterative scheduling strategies (iterative-ilp / -minreg / -maxocc)
# and max-ILP with relaxed occupancy, against the tree's max-ILP build,
# interleaved three times at 200 steps.
set -u
O=gpurun_out/r3v4
mkdir -p $O
run() {  # run VARIANT TAG ARGS...
  local v=$1 tag=$2; shift 2
  local L=""
  [ "$v" != new ] && L=build_v/$v/librtamd.so
  RTAMD_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie "$@" > $O/$tag.json 2> $O/$tag.err || exit $?
}
for rep in a b c; do
  for v in new itilp itmin itocc ilprel; do run $v ${v}_$rep --steps 200; done
done
echo done > $O/done.txt
