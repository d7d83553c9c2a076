#!/bin/bash
# Round-5 BASELINE shapes on one MI355X: the 1M headline config, the 500-iteration headline
# average, LambdaRank 5M x 300, regression EFB + GOSS 12.5M x 500 (GOSS active: 12 warmup
# iterations) serial fp / quantized and voting on a one-rank communicator. Each step has its own
# limit; the first failure ends it.
set -u
OUT=${1:-gpurun_out/shapes}
mkdir -p $OUT
export TMPDIR=/tmp
( while true; do date > $OUT/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "=== $name" >> $OUT/steps.log
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $OUT/steps.log
  grep -E "^\{" $OUT/$name.log | cut -c1-420 >> $OUT/steps.log
  [ $rc -eq 0 ] || exit $rc
}
run h1m 300 python bench.py --rows 1000000 --steps 50 --warmup 5
run h500 400 python bench.py --steps 500 --warmup 5
run ltr5m 600 python scripts/bench_suite.py --config ltr --rows 5000000 --features 300 --steps 20 --warmup 3
run goss12 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 10 --warmup 12
run goss12q 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 10 --warmup 12 --quantized
run vote12 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --learner voting --steps 10 --warmup 12
run pltr 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/pltr -o run -- python3 scripts/bench_suite.py --config ltr --rows 5000000 --features 300 --steps 10 --warmup 3
python scripts/prof_summary.py $OUT/pltr "LambdaRank 5M x 300, 255 leaves" 13 > $OUT/pltr_summary.md 2>&1; rm -rf $OUT/pltr
run pgoss 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/pgoss -o run -- python3 scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 10 --warmup 12
python scripts/prof_summary.py $OUT/pgoss "regression EFB + GOSS 12.5M x 500, 255 leaves, fp" 22 > $OUT/pgoss_summary.md 2>&1; rm -rf $OUT/pgoss
