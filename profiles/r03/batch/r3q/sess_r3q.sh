# r3q: rank 0's piece weight with order_split 15 (N = 8, 4, 2 emulated), and
# whether clean learning (learn_alone) or walk-length costs (learn_cost 0)
# change the pieces' order.
set -u
O=gpurun_out/r3q
mkdir -p $O
b() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie "$@" > $O/$tag.json 2> $O/$tag.err || exit $?; }
e() { local tag=$1 n=$2 r=$3; shift 3; bash tools/emulate.sh $O/emu $tag $n "$r" --warmup 5 --partition pieces "$@" || exit $?; }
b base200
b base20 --steps 20
e w60 8 "0 1" --steps 200 --root-weight 0.6 --set order_split=15
e w65 8 "0 1" --steps 200 --root-weight 0.65 --set order_split=15
e w70 8 "0 1" --steps 200 --root-weight 0.7 --set order_split=15
e w65_20 8 "0 1 7" --steps 20 --root-weight 0.65 --set order_split=15
e w60_20 8 "0 1" --steps 20 --root-weight 0.6 --set order_split=15
e alone 8 "1" --steps 200 --root-weight 0.65 --set order_split=0,learn_alone=1
e alone15 8 "1" --steps 200 --root-weight 0.65 --set order_split=15,learn_alone=1
e cost0 8 "1" --steps 200 --root-weight 0.65 --set order_split=0,learn_cost=0
e w75_20 4 "0 1" --steps 20 --root-weight 0.75 --set order_split=15
e w85_20 4 "0 1" --steps 20 --root-weight 0.85 --set order_split=15
e w100_20 2 "0 1" --steps 20 --root-weight 1.0 --set order_split=15
e w90_20 2 "0 1" --steps 20 --root-weight 0.9 --set order_split=15
e w100_20_alone 2 "0 1" --steps 20 --root-weight 1.0 --set order_split=15,learn_alone=1
e w100_20_f4 2 "0 1" --steps 20 --root-weight 1.0 --set order_split=15 --batch 4
e w100_200 2 "0 1" --steps 200 --root-weight 1.0 --set order_split=15
e asmn_w65 8 "0" --steps 200 --root-weight 0.65 --set order_split=15 --assembly-priority normal
e asmn_w65_20 8 "0" --steps 20 --root-weight 0.65 --set order_split=15 --assembly-priority normal
e asmn_w80 8 "0" --steps 200 --root-weight 0.8 --set order_split=15 --assembly-priority normal
bash tools/rehearse.sh $O/rehearse 8 pieces --steps 20 --warmup 5 --root-weight 0.65 --set order_split=15 --assembly-priority normal || exit $?
echo done > $O/done.txt
