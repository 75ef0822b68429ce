set -u
OUT=gpurun_out/warm; mkdir -p $OUT
for rep in 1 2; do
for sw in "20 5" "20 100" "100 5" "20 400"; do set -- $sw
  timeout -k 10 120 python bench.py --steps $1 --warmup $2 --no-cpu-baseline > $OUT/s$1_w$2_$rep.json 2>/dev/null || exit 1
done; done
