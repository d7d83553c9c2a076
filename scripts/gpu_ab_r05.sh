#!/bin/bash
# Paired A/B of an env-selected variant against the default on one box (headline 10M and 1.25M),
# alternating A B A B so drift shows. Usage: scripts/gpu_ab_r05.sh <outdir> "<ENV=VAL ...>"
set -u
OUT=${1:-gpurun_out/ab}
VAR=${2:-}
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
  grep -E "^\{|fstamps (partition|hist)|frontier:" $OUT/$name.log | cut -c1-200 >> $OUT/steps.log
  [ $rc -eq 0 ] || exit $rc
}
for i in 1 2; do
  run a10_$i 300 python bench.py --steps 40 --warmup 5
  run b10_$i 300 env $VAR python bench.py --steps 40 --warmup 5
done
for i in 1 2; do
  run a1_$i 300 python bench.py --rows 1250000 --steps 50 --warmup 5
  run b1_$i 300 env $VAR python bench.py --rows 1250000 --steps 50 --warmup 5
done
LGAP_FSTAMPS=1 run sa 300 python bench.py --steps 10 --warmup 1
LGAP_FSTAMPS=1 run sb 300 env $VAR python bench.py --steps 10 --warmup 1
