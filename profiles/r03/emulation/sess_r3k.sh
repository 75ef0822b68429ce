# r3k: the final N > 1 defaults (weak scaling, bands, 4 launches in flight x N
# frames, one exchange per 4 launches) emulated rank by rank, and rehearsed
# with gloo ranks sharing the GPU (frames verified).
set -u
O=gpurun_out/r3k
mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcie > $O/base20.json 2> $O/base20.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie > $O/base200.json 2> $O/base200.err || exit $?
e() { local tag=$1 n=$2 r=$3; shift 3; bash tools/emulate.sh $O/emu $tag $n "$r" --warmup 5 "$@" || exit $?; }
e w20 8 "0 1 7" --steps 20
e w200 8 "0 1 7" --steps 200
e w20 4 "0 1 3" --steps 20
e w20 2 "0 1" --steps 20
e s20 8 "0 1 7" --steps 20 --scaling strong
e s200 8 "0 1" --steps 200 --scaling strong
e s20 4 "0 1" --steps 20 --scaling strong
bash tools/rehearse.sh $O/rehearse 2 bands --steps 20 --warmup 5 || exit $?
bash tools/rehearse.sh $O/rehearse 4 bands --steps 20 --warmup 5 || exit $?
bash tools/rehearse.sh $O/rehearse 8 bands --steps 20 --warmup 5 || exit $?
bash tools/rehearse.sh $O/rehearse 4 tiles --steps 20 --warmup 5 --gather radiance || exit $?
mkdir -p $O/rehearse_strong
bash tools/rehearse.sh $O/rehearse_strong 8 bands --steps 20 --warmup 5 --scaling strong --gather radiance || exit $?
echo done > $O/done.txt
