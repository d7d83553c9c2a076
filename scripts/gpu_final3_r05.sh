#!/bin/bash
# Round-5 final pass, part 2: the wide BASELINE shapes and the 500-iteration lines.
set -u
OUT=${1:-gpurun_out/final3}
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
run h500 400 python bench.py --steps 500 --warmup 5
run l255 400 python bench.py --num-leaves 255 --steps 500 --warmup 5
run ltr5m 600 python scripts/bench_suite.py --config ltr --rows 5000000 --features 300 --steps 20 --warmup 3
run goss12 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 10 --warmup 12
run goss12q 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 10 --warmup 12 --quantized
run vote12 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --learner voting --steps 10 --warmup 12
