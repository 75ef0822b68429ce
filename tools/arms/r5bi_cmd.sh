set -u
O=gpurun_out/r5bi; mkdir -p $O
for rep in 1 2; do
  bash tools/emulate.sh $O/emu nccl_rep$rep 8 "1" --steps 20 --warmup 5 || exit $?
  BENCH_DIST_BACKEND=gloo bash tools/emulate.sh $O/emu gloo_rep$rep 8 "1" --steps 20 --warmup 5 || exit $?
  BENCH_EMULATE_NOX=1 bash tools/emulate.sh $O/emu nox_rep$rep 8 "1" --steps 20 --warmup 5 || exit $?
done
