# r3l: weak scaling with rotating contiguous pieces (--partition pieces,
# rt_render_batch_lists_device) against the weighted interleaved bands,
# emulated rank by rank on one GPU; gloo rehearsals check the frames.
set -u
O=gpurun_out/r3l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -rA --timeout 300 --timeout-method thread \
  -k "pieces or batch or async" > $O/pytest_pieces.log 2>&1 || exit $?
timeout -k 10 300 python tools/pipeline_bench.py --slots 4 --frames 400 > $O/pipeline.jsonl 2> $O/pipeline.err || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20_pcie.json 2> $O/bench20_pcie.err || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcie > $O/base20.json 2> $O/base20.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie > $O/base200.json 2> $O/base200.err || exit $?
e() { local tag=$1 n=$2 r=$3; shift 3; bash tools/emulate.sh $O/emu $tag $n "$r" --warmup 5 "$@" || exit $?; }
e p20 8 "0 1 7" --steps 20 --partition pieces
e b20 8 "0 1 7" --steps 20 --partition bands
e p200 8 "0 1" --steps 200 --partition pieces
e b200 8 "0 1" --steps 200 --partition bands
e p20 4 "0 1" --steps 20 --partition pieces
e b20 4 "0 1" --steps 20 --partition bands
e p20 2 "0 1" --steps 20 --partition pieces
e b20 2 "0 1" --steps 20 --partition bands
bash tools/rehearse.sh $O/rehearse 8 pieces --steps 20 --warmup 5 || exit $?
bash tools/rehearse.sh $O/rehearse 4 pieces --steps 20 --warmup 5 --gather radiance || exit $?
bash tools/rehearse.sh $O/rehearse 2 pieces --steps 20 --warmup 5 || exit $?
bash tools/rehearse.sh $O/rehearse 8 bands --steps 20 --warmup 5 || exit $?
bash tools/rehearse.sh $O/rehearse 4 tiles --steps 20 --warmup 5 --gather radiance || exit $?
echo done > $O/done.txt
