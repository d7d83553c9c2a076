#!/bin/bash
# Full GPU suite on the working tree, then A (variants/lib_lambdagap.so) vs the working tree at 10M
# and 1.25M, alternating twice. Each step has its own limit; the first failure ends it.
set -u
OUT=${1:-gpurun_out/final}
mkdir -p $OUT
export TMPDIR=/tmp
( while true; do date > $OUT/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
A=$PWD/variants/lib_lambdagap.so
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "=== $name" >> $OUT/steps.log
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $OUT/steps.log
  grep -E "^\{|passed|failed" $OUT/$name.log | cut -c1-190 >> $OUT/steps.log
  [ $rc -eq 0 ] || exit $rc
}
run gputests 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread
for i in 1 2; do
  run A10_$i 300 env LAMBDAGAP_LIB=$A python bench.py --steps 40 --warmup 5
  run C10_$i 300 python bench.py --steps 40 --warmup 5
  run A1_$i 300 env LAMBDAGAP_LIB=$A python bench.py --rows 1250000 --steps 50 --warmup 5
  run C1_$i 300 python bench.py --rows 1250000 --steps 50 --warmup 5
done
run Cdrv 300 python bench.py --gpus 1 --steps 20 --warmup 5
