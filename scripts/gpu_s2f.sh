#!/bin/bash
# CEGB coupled penalties on the device + frontier parity subset; GOSS 12.5M x 500 A/B against
# the session-start library (ab_lib/, LAMBDAGAP_LIB)
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_learner.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "cegb or frontier_engine or forced_splits_on or host_policy" > $OUT/tc.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" $OUT/tc.log | tail -40
[ $rc -ne 0 ] && exit $rc
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -E "^\{" $OUT/$name.log | tail -1 | cut -c1-300
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
LAMBDAGAP_LIB=$PWD/ab_lib/lib_lambdagap_266d1bc.so run goss_old 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 20 --warmup 12
run goss_new 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 20 --warmup 12
