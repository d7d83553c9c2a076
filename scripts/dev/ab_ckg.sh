# A/B of the select's compact candidate table (default) against reading the full keys (select_ckg=0)
set -u
OUT=gpurun_out/ab_ckg
mkdir -p $OUT
for v in 1 0 1 0; do
  if [ $v = 0 ]; then export LGAP_KERNEL=select_ckg=0; else unset LGAP_KERNEL; fi
  timeout -k 10 200 python3 scripts/bench_suite.py --config regression_goss --rows 3000000 --features 500 --steps 20 --warmup 11 > $OUT/goss_$v.log 2>&1 || exit 1
  timeout -k 10 200 python3 scripts/bench_suite.py --config ltr --rows 2000000 --features 300 --steps 20 --warmup 3 > $OUT/ltr_$v.log 2>&1 || exit 1
  timeout -k 10 200 python3 bench.py --steps 30 --warmup 3 > $OUT/b10_$v.log 2>&1 || exit 1
  echo "ckg=$v goss3m $(grep -o '"value": [0-9.]*' $OUT/goss_$v.log) ltr2m $(grep -o '"value": [0-9.]*' $OUT/ltr_$v.log) 10M $(grep -o '"value": [0-9.]*' $OUT/b10_$v.log)"
done
