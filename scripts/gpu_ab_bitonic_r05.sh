#!/bin/bash
# select bitonic network with wave barriers for in-segment steps (working tree) vs the previous
# commit (variants/lib_h.so): 255-leaf shapes (alive lists > 256 nodes) and the headline
set -u
OUT=${1:-gpurun_out/abbit}
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
  grep -E "^\{|passed|failed|fstamps select" $OUT/$name.log | cut -c1-200 >> $OUT/steps.log
  [ $rc -eq 0 ] || exit $rc
}
run kt 500 python -u -m pytest tests/test_gpu_learner.py -x -q --timeout 200 --timeout-method thread -k "speculation or frontier or goss or cegb or quantized or forced or lambdarank"
for i in 1 2; do
  run Agoss_$i 400 env LAMBDAGAP_LIB=$A python scripts/bench_suite.py --config regression_goss --rows 3000000 --features 500 --steps 10 --warmup 12
  run Cgoss_$i 400 python scripts/bench_suite.py --config regression_goss --rows 3000000 --features 500 --steps 10 --warmup 12
  run A255_$i 300 env LAMBDAGAP_LIB=$A python bench.py --num-leaves 255 --steps 100 --warmup 5
  run C255_$i 300 python bench.py --num-leaves 255 --steps 100 --warmup 5
done
run Cst 300 env LGAP_FSTAMPS=1 python scripts/bench_suite.py --config regression_goss --rows 3000000 --features 500 --steps 5 --warmup 12
