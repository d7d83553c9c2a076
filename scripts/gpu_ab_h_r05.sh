#!/bin/bash
# A (variants/lib_a2.so, previous commit) vs the working tree: reduce tiles in LDS + a 4x-CU reduce
# grid. LambdaRank 2M x 300 (many reduce items per block) and the 10M / 1.25M headline.
set -u
OUT=${1:-gpurun_out/abred}
mkdir -p $OUT
export TMPDIR=/tmp
( while true; do date > $OUT/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
A=$PWD/variants/lib_h.so
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "=== $name" >> $OUT/steps.log
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $OUT/steps.log
  grep -E "^\{|passed|failed|fstamps (hist|partition) |chain" $OUT/$name.log | cut -c1-190 >> $OUT/steps.log
  [ $rc -eq 0 ] || exit $rc
}
run kt 300 python -u -m pytest tests/test_frontier_kernels.py -x -q --timeout 150 --timeout-method thread
for i in 1 2; do
  run Altr_$i 400 env LAMBDAGAP_LIB=$A python scripts/bench_suite.py --config ltr --rows 2000000 --features 300 --steps 10 --warmup 3
  run Cltr_$i 400 python scripts/bench_suite.py --config ltr --rows 2000000 --features 300 --steps 10 --warmup 3
  run A10_$i 300 env LAMBDAGAP_LIB=$A python bench.py --steps 40 --warmup 5
  run C10_$i 300 python bench.py --steps 40 --warmup 5
  run A1_$i 300 env LAMBDAGAP_LIB=$A python bench.py --rows 1250000 --steps 50 --warmup 5
  run C1_$i 300 python bench.py --rows 1250000 --steps 50 --warmup 5
done
run Cst 300 env LGAP_FSTAMPS=1 python bench.py --steps 10 --warmup 1
