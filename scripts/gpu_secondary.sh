#!/bin/bash
# Secondary BASELINE configs + 255-leaf headline, frontier engine vs the sequential chain.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
export LGAP_FRONTIER_STATS=1
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -E "frontier:|^\{" $OUT/$name.log | tail -2 | cut -c1-400
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
run b255 300 python bench.py --num-leaves 255 --steps 30 --warmup 3
LGAP_FRONTIER=0 run b255seq 300 python bench.py --num-leaves 255 --steps 30 --warmup 3
run ltr5 400 python scripts/bench_suite.py --config ltr --rows 5000000 --features 300 --steps 20 --warmup 3
LGAP_FRONTIER=0 run ltr5seq 400 python scripts/bench_suite.py --config ltr --rows 5000000 --features 300 --steps 20 --warmup 3
run goss12 600 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 20 --warmup 12
LGAP_FRONTIER=0 run goss12seq 600 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 20 --warmup 12
