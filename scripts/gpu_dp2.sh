#!/bin/bash
# DP caps: rehearsals + single-rank RCCL bench with stats; quantized tests (k_qmax)
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_learner.py -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -k "data_parallel or quantized" > $OUT/dp.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/dp.log | tail -25; [ $rc -ne 0 ] && exit $rc
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -E "^\{|frontier:" $OUT/$name.log | tail -2 | cut -c1-300
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
export LGAP_FRONTIER_STATS=1
run dp10 300 python bench.py --rehearse-dp --steps 30 --warmup 3
LGAP_FRONTIER_KCAP=off run dp10nc 300 python bench.py --rehearse-dp --steps 30 --warmup 3
run dp1 300 python bench.py --rehearse-dp --rows 1250000 --steps 50 --warmup 3
run b10q 300 python bench.py --steps 30 --warmup 3 --quantized
