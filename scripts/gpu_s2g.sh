#!/bin/bash
# after removing the row-per-thread path (k_f_hist registers back to the session-start shape)
# and templating the select on CEGB: CEGB / frontier tests, GOSS 12.5M x 500, headline lines
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_learner.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "cegb or frontier_engine or forced_splits_on or host_policy or quantized or bagging" > $OUT/tc.log 2>&1 || { tail -30 $OUT/tc.log; exit 1; }
tail -1 $OUT/tc.log
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -E "^\{" $OUT/$name.log | tail -1 | cut -c1-400
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
run goss12 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 20 --warmup 12
run goss12q 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 20 --warmup 12 --quantized
run b10 300 python bench.py --steps 40 --warmup 3
run b1 300 python bench.py --rows 1250000 --steps 50 --warmup 5
run b10q 300 python bench.py --steps 40 --warmup 3 --quantized
