#!/bin/bash
# Three-way paired A/B on one box: A = variants/lib_lambdagap.so (previous commit), B =
# variants/lib_b.so, C = the working tree's library; alternating A B C twice at 10M and 1.25M,
# then one LambdaRank 2M x 300 line each and per-round stamps of C.
set -u
OUT=${1:-gpurun_out/ab3}
mkdir -p $OUT
export TMPDIR=/tmp
( while true; do date > $OUT/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
A=$PWD/variants/lib_lambdagap.so
B=$PWD/variants/lib_b.so
C=$PWD/lambdagap_amd/lib/lib_lambdagap.so
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "=== $name" >> $OUT/steps.log
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $OUT/steps.log
  grep -E "^\{|fstamps (scan|select|hist) " $OUT/$name.log | cut -c1-190 >> $OUT/steps.log
  [ $rc -eq 0 ] || exit $rc
}
for i in 1 2; do
  for v in A B C; do
    eval L=\$$v
    run ${v}10_$i 300 env LAMBDAGAP_LIB=$L python bench.py --steps 40 --warmup 5
  done
done
for i in 1 2; do
  for v in A B C; do
    eval L=\$$v
    run ${v}1_$i 300 env LAMBDAGAP_LIB=$L python bench.py --rows 1250000 --steps 50 --warmup 5
  done
done
for v in A C; do
  eval L=\$$v
  run ${v}ltr 400 env LAMBDAGAP_LIB=$L python scripts/bench_suite.py --config ltr --rows 2000000 --features 300 --steps 10 --warmup 3
done
run Cst 300 env LGAP_FSTAMPS=1 python bench.py --steps 10 --warmup 1
