# r3r: the exchange at the end of a 20-step run (pieces, w 0.7, order_split 15):
# exchange every 4 launches (G 32) or 2 (G 16); senders' copies at normal
# priority (--exchange-priority 2); N = 8 / 4 / 2 emulated.
set -u
O=gpurun_out/r3r
mkdir -p $O
b() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie "$@" > $O/$tag.json 2> $O/$tag.err || exit $?; }
e() { local tag=$1 n=$2 r=$3; shift 3; bash tools/emulate.sh $O/emu $tag $n "$r" --warmup 5 --partition pieces --set order_split=15 "$@" || exit $?; }
b base20_1 --steps 20
b base20_2 --steps 20
b base200
e g32 8 "0 1 7" --steps 20 --root-weight 0.7
e g16 8 "0 1 7" --steps 20 --root-weight 0.7 --exchange-every 16
e g32p2 8 "0 1 7" --steps 20 --root-weight 0.7 --exchange-priority 2
e g16p2 8 "0 1" --steps 20 --root-weight 0.7 --exchange-every 16 --exchange-priority 2
e g32p2_200 8 "0 1" --steps 200 --root-weight 0.7 --exchange-priority 2
e n4g16 4 "0 1" --steps 20 --root-weight 0.75 --exchange-every 8
e n4g16 4 "0 1" --steps 20 --root-weight 0.75 --exchange-every 16
e n4p2 4 "0 1" --steps 20 --root-weight 0.75 --exchange-priority 2
e n2p2 2 "0 1" --steps 20 --root-weight 1.0 --exchange-priority 2
e n2g4 2 "0 1" --steps 20 --root-weight 1.0 --exchange-every 4
echo done > $O/done.txt
