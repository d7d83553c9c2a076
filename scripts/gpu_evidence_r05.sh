#!/bin/bash
# closing evidence: quantized and 15-bin (4-bit rows) headline variants, the owner-computes
# rehearsal at 10M, kernel profiles of the wide shapes at the round's final code
set -u
OUT=${1:-gpurun_out/evidence}
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
  grep -E "^\{" $OUT/$name.log | cut -c1-330 >> $OUT/steps.log
  [ $rc -eq 0 ] || exit $rc
}
run quant 300 python bench.py --steps 40 --warmup 5 --quantized
run bins15 300 python bench.py --steps 40 --warmup 5 --max-bin 15
run owner10m 300 python bench.py --steps 40 --warmup 5 --rehearse-dp
run pltr 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/pltr -o run -- python3 scripts/bench_suite.py --config ltr --rows 5000000 --features 300 --steps 10 --warmup 3
python scripts/prof_summary.py $OUT/pltr "LambdaRank 5M x 300, 255 leaves (round-5 final)" 13 > $OUT/pltr_summary.md 2>&1; rm -rf $OUT/pltr
run pgoss 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/pgoss -o run -- python3 scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 10 --warmup 12
python scripts/prof_summary.py $OUT/pgoss "regression EFB + GOSS 12.5M x 500, 255 leaves, fp (round-5 final)" 22 > $OUT/pgoss_summary.md 2>&1; rm -rf $OUT/pgoss
