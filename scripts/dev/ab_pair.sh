# A/B of the serial pair-best ahead of the select (default on wide data) against phase A over all keys
set -u
OUT=gpurun_out/ab_pair
mkdir -p $OUT
for v in 1 0 1 0; do
  export LGAP_KERNEL=pair_best=$v
  timeout -k 10 200 python3 scripts/bench_suite.py --config regression_goss --rows 3000000 --features 500 --steps 20 --warmup 11 > $OUT/goss_$v.log 2>&1 || exit 1
  echo "goss3m pair=$v $(tail -1 $OUT/goss_$v.log | cut -c1-130)"
  timeout -k 10 200 python3 scripts/bench_suite.py --config ltr --rows 2000000 --features 300 --steps 20 --warmup 3 > $OUT/ltr_$v.log 2>&1 || exit 1
  echo "ltr2m pair=$v $(tail -1 $OUT/ltr_$v.log | cut -c1-130)"
done
