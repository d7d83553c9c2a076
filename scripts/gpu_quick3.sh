#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
export LGAP_FRONTIER_STATS=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "wide_rows or frontier_engine or first_tree or validation_scoring or categorical" > $OUT/t.log 2>&1; rc=$?
tail -3 $OUT/t.log; [ $rc -ne 0 ] && exit $rc
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -E "fstamps select|frontier:|^\{" $OUT/$name.log | tail -2 | cut -c1-300
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
LGAP_FSTAMPS=1 run gst 300 python scripts/bench_suite.py --config regression_goss --rows 2000000 --features 500 --steps 3 --warmup 12
run goss12 600 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 20 --warmup 12
run b10 300 python bench.py --steps 30 --warmup 3
run b255 300 python bench.py --num-leaves 255 --steps 30 --warmup 3
