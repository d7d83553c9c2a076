#!/bin/bash
# Round-5 closing pass: full GPU suite, smoke, the driver's bench line, the wide shapes after the
# last select change. Each step has its own limit; the first failure ends it.
set -u
OUT=${1:-gpurun_out/final4}
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
  grep -E "^\{|passed|failed|smoke ok" $OUT/$name.log | cut -c1-330 >> $OUT/steps.log
  [ $rc -eq 0 ] || exit $rc
}
run gputests 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
run bench_b 300 python bench.py --gpus 1 --steps 20 --warmup 5
run ltr5m 600 python scripts/bench_suite.py --config ltr --rows 5000000 --features 300 --steps 20 --warmup 3
run goss12 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 10 --warmup 12
run vote12 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --learner voting --steps 10 --warmup 12
