#!/bin/bash
# round-3 secondary BASELINE configurations on the current code (one GPU): EFB + GOSS
# 12.5M x 500 (serial, quantized, voting), 255 leaves x 500 iterations, LambdaRank 5M x 300
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -E "^\{" $OUT/$name.log | tail -1 | cut -c1-600
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
run goss12 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 20 --warmup 3
run goss12q 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 20 --warmup 3 --quantized
run vote12 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --learner voting --steps 20 --warmup 3
run b255 600 python bench.py --num-leaves 255 --steps 500 --warmup 5
run ltr 600 python scripts/bench_suite.py --config ltr --rows 5000000 --steps 20 --warmup 5
