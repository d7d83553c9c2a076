# A/B of the select's merged alive order (default) against the full re-sort (select_merge=0)
set -u
OUT=gpurun_out/ab_merge
mkdir -p $OUT
for v in 1 0 1 0; do
  if [ $v = 0 ]; then export LGAP_KERNEL=select_merge=0; else unset LGAP_KERNEL; fi
  timeout -k 10 200 python3 scripts/bench_suite.py --config regression_goss --rows 3000000 --features 500 --steps 20 --warmup 11 > $OUT/goss_$v.log 2>&1 || exit 1
  echo "goss3m merge=$v $(tail -1 $OUT/goss_$v.log | cut -c1-160)"
  timeout -k 10 200 python3 bench.py --num-leaves 255 --steps 30 --warmup 3 > $OUT/b255_$v.log 2>&1 || exit 1
  echo "10M-255 merge=$v $(tail -1 $OUT/b255_$v.log | cut -c1-120)"
done
