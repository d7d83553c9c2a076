#!/bin/bash
# Paired A/B of the working tree's library (B) against variants/lib_lambdagap.so (A, the previous
# commit's build) on one box, alternating A B A B; 10M headline, 1.25M, and (wide data) LambdaRank 2M.
set -u
OUT=${1:-gpurun_out/abl}
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
  grep -E "^\{|fstamps scan" $OUT/$name.log | cut -c1-200 >> $OUT/steps.log
  [ $rc -eq 0 ] || exit $rc
}
for i in 1 2; do
  run a10_$i 300 env LAMBDAGAP_LIB=$A python bench.py --steps 40 --warmup 5
  run b10_$i 300 python bench.py --steps 40 --warmup 5
done
for i in 1 2; do
  run a1_$i 300 env LAMBDAGAP_LIB=$A python bench.py --rows 1250000 --steps 50 --warmup 5
  run b1_$i 300 python bench.py --rows 1250000 --steps 50 --warmup 5
done
run altr 400 env LAMBDAGAP_LIB=$A python scripts/bench_suite.py --config ltr --rows 2000000 --features 300 --steps 10 --warmup 3
run bltr 400 python scripts/bench_suite.py --config ltr --rows 2000000 --features 300 --steps 10 --warmup 3
run sa 300 env LGAP_FSTAMPS=1 LAMBDAGAP_LIB=$A python bench.py --rows 1250000 --steps 10 --warmup 1
run sb 300 env LGAP_FSTAMPS=1 python bench.py --rows 1250000 --steps 10 --warmup 1
