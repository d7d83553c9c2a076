#!/bin/bash
# paired A/B of env settings on LambdaRank 5M x 300 and GOSS 12.5M x 500
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
one() {
  env $1 timeout -k 10 300 python scripts/bench_suite.py --config ltr --rows 5000000 --steps 10 --warmup 5 > $OUT/abw.log 2>&1 || exit $?
  echo "=== LTR $1"; grep -E "^\{" $OUT/abw.log | cut -c1-120
  env $1 timeout -k 10 300 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 10 --warmup 12 > $OUT/abw.log 2>&1 || exit $?
  echo "=== GOSS $1"; grep -E "^\{" $OUT/abw.log | cut -c1-120
}
one "X=1"
for ab in "$@"; do one "$ab"; done
