#!/bin/bash
# Data / feature / voting parallel on the frontier: the multi-rank rehearsals (tree-for-tree
# equality with the host learners), the one-rank owner-computes and all-reduce rehearsals and the
# serial frontier at 1.25M and 10M. Each step has its own limit; the first failure ends it.
set -u
OUT=${1:-gpurun_out/dp}
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
  grep -E "^\{|passed|failed|error" $OUT/$name.log | cut -c1-330 >> $OUT/steps.log
  [ $rc -eq 0 ] || exit $rc
}
run tests 600 python -u -m pytest tests/test_gpu_learner.py -x -q --timeout 300 --timeout-method thread -k "parallel or rehearsal"
run serial_1p25 300 python bench.py --rows 1250000 --steps 50 --warmup 5
run owner_1p25 300 python bench.py --rows 1250000 --steps 50 --warmup 5 --rehearse-dp
LGAP_DP_TRANSPORT=allreduce run allreduce_1p25 300 python bench.py --rows 1250000 --steps 50 --warmup 5 --rehearse-dp
run serial_10m 300 python bench.py --steps 40 --warmup 3
run owner_10m 300 python bench.py --steps 40 --warmup 3 --rehearse-dp
