# A/B of the frontier's speculation budget (LGAP_FRONTIER_SPEC alpha) at the headline shapes
set -u
OUT=gpurun_out/ab_alpha
mkdir -p $OUT
for rep in 1 2; do
for a in ${ALPHAS:-fixed 1.5 2 3}; do
  LGAP_FRONTIER_SPEC=$a timeout -k 10 200 python3 bench.py --steps 30 --warmup 3 > $OUT/b10_$a.log 2>&1 || exit 1
  LGAP_FRONTIER_SPEC=$a timeout -k 10 200 python3 bench.py --rows 1250000 --steps 50 --warmup 5 > $OUT/b1_$a.log 2>&1 || exit 1
  echo "alpha=$a 10M $(grep -o '"value": [0-9.]*' $OUT/b10_$a.log) 1.25M $(grep -o '"value": [0-9.]*' $OUT/b1_$a.log)"
done
done
