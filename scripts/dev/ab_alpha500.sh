# speculation budget (LGAP_FRONTIER_SPEC alpha) over 500 iterations at 10M x 28 / 63 leaves
set -u
OUT=gpurun_out/ab_alpha500
mkdir -p $OUT
for rep in 1 2; do
for a in ${ALPHAS:-0.75 fixed 1.25 1.5}; do
  LGAP_FRONTIER_SPEC=$a timeout -k 10 200 python3 bench.py --steps 500 --warmup 3 > $OUT/b10_$a.log 2>&1 || exit 1
  echo "alpha=$a 10M/500 $(grep -o '"value": [0-9.]*' $OUT/b10_$a.log)"
done
done
