#!/bin/bash
# Round-5 measurement pass (one gpurun call): LambdaRank kernel before/after, owner-computes DP
# rehearsal vs all-reduce vs serial, frontier voting vs serial on the wide GOSS shape, the
# 500-iteration headline average. Every step has its own time limit; the first failure ends it.
set -u
OUT=gpurun_out/r05m
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
  tail -3 $OUT/$name.log | cut -c1-400 >> $OUT/steps.log
  [ $rc -eq 0 ] || exit $rc
}
HEADLIB=$PWD/variants/lib_head.so
run ltr_prof_new 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/pltr_new -o run -- python3 scripts/bench_suite.py --config ltr --rows 2000000 --features 300 --steps 5 --warmup 1
python scripts/prof_summary.py $OUT/pltr_new "LambdaRank 2M x 300 (new kernel)" 6 > $OUT/pltr_new_summary.md; rm -rf $OUT/pltr_new
if [ -f $HEADLIB ]; then
  LAMBDAGAP_LIB=$HEADLIB run ltr_prof_old 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/pltr_old -o run -- python3 scripts/bench_suite.py --config ltr --rows 2000000 --features 300 --steps 5 --warmup 1
  python scripts/prof_summary.py $OUT/pltr_old "LambdaRank 2M x 300 (round-4 kernel)" 6 > $OUT/pltr_old_summary.md; rm -rf $OUT/pltr_old
fi
run ltr5m 600 python scripts/bench_suite.py --config ltr --rows 5000000 --features 300 --steps 20 --warmup 3
run dp_owner_1p25 300 python bench.py --rows 1250000 --steps 50 --warmup 5 --rehearse-dp
LGAP_DP_TRANSPORT=allreduce run dp_allreduce_1p25 300 python bench.py --rows 1250000 --steps 50 --warmup 5 --rehearse-dp
run serial_1p25 300 python bench.py --rows 1250000 --steps 50 --warmup 5
run dp_owner_10m 300 python bench.py --steps 40 --warmup 3 --rehearse-dp
LGAP_DP_TRANSPORT=allreduce run dp_allreduce_10m 300 python bench.py --steps 40 --warmup 3 --rehearse-dp
run headline_500 400 python bench.py --steps 500 --warmup 5
run vote12 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --learner voting --steps 20 --warmup 3
run serial12 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 20 --warmup 3
