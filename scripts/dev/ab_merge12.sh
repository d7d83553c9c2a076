set -u
OUT=gpurun_out/ab_merge12
mkdir -p $OUT
for v in 1 0 1 0; do
  if [ $v = 0 ]; then export LGAP_KERNEL=select_merge=0; else unset LGAP_KERNEL; fi
  timeout -k 10 300 python3 scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 20 --warmup 12 > $OUT/g_$v.log 2>&1 || exit 1
  echo "goss12.5m merge=$v $(grep -o '"value": [0-9.]*' $OUT/g_$v.log)"
done
