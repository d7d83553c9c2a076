#!/bin/bash
# select rank sort up to 512 alive nodes (B, variants/lib_r512.so) vs the bitonic network beyond 256
# (A, the working tree) on the 255-leaf shapes
set -u
OUT=${1:-gpurun_out/abrank}
mkdir -p $OUT
export TMPDIR=/tmp
( while true; do date > $OUT/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
B=$PWD/variants/lib_r512.so
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "=== $name" >> $OUT/steps.log
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $OUT/steps.log
  grep -E "^\{" $OUT/$name.log | cut -c1-200 >> $OUT/steps.log
  [ $rc -eq 0 ] || exit $rc
}
for i in 1 2; do
  run Altr_$i 400 python scripts/bench_suite.py --config ltr --rows 2000000 --features 300 --steps 10 --warmup 3
  run Bltr_$i 400 env LAMBDAGAP_LIB=$B python scripts/bench_suite.py --config ltr --rows 2000000 --features 300 --steps 10 --warmup 3
  run Agoss_$i 400 python scripts/bench_suite.py --config regression_goss --rows 3000000 --features 500 --steps 10 --warmup 12
  run Bgoss_$i 400 env LAMBDAGAP_LIB=$B python scripts/bench_suite.py --config regression_goss --rows 3000000 --features 500 --steps 10 --warmup 12
  run A255_$i 300 python bench.py --num-leaves 255 --steps 100 --warmup 5
  run B255_$i 300 env LAMBDAGAP_LIB=$B python bench.py --num-leaves 255 --steps 100 --warmup 5
done
