# closing evidence of round 6: the README performance table's lines on one box
set -u
OUT=gpurun_out/final
mkdir -p $OUT
line() { echo "$1 $(grep -o '"value": [0-9.]*' $2 | head -1) $(grep -o '"auc": [0-9.]*' $2 | head -1)"; }
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $OUT/b10_20.log 2>&1 || exit 1; line "10M 63L 20 steps" $OUT/b10_20.log
timeout -k 10 200 python3 bench.py --steps 40 --warmup 3 > $OUT/b10_40.log 2>&1 || exit 1; line "10M 63L 40 steps" $OUT/b10_40.log
timeout -k 10 200 python3 bench.py --steps 500 --warmup 0 > $OUT/b10_500.log 2>&1 || exit 1; line "10M 63L 500 iterations" $OUT/b10_500.log
timeout -k 10 200 python3 bench.py --rows 1000000 --steps 50 --warmup 5 > $OUT/b1m.log 2>&1 || exit 1; line "1M 63L 50 steps" $OUT/b1m.log
timeout -k 10 200 python3 bench.py --rows 1250000 --steps 50 --warmup 5 > $OUT/b125.log 2>&1 || exit 1; line "1.25M 63L 50 steps" $OUT/b125.log
timeout -k 10 300 python3 bench.py --num-leaves 255 --steps 500 --warmup 0 > $OUT/b10_255.log 2>&1 || exit 1; line "10M 255L 500 iterations" $OUT/b10_255.log
timeout -k 10 300 python3 scripts/bench_suite.py --config ltr --rows 5000000 --features 300 --steps 20 --warmup 3 > $OUT/ltr5m.log 2>&1 || exit 1; line "LambdaRank 5M x 300" $OUT/ltr5m.log
timeout -k 10 300 python3 scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 20 --warmup 12 > $OUT/goss12m.log 2>&1 || exit 1; line "GOSS 12.5M x 500" $OUT/goss12m.log
