#!/bin/bash
# select phases of the 255-leaf shapes (in-kernel stamps): GOSS 3M x 500 and LambdaRank 2M x 300
set -u
OUT=${1:-gpurun_out/sel255}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 env LGAP_FSTAMPS=1 python scripts/bench_suite.py --config regression_goss --rows 3000000 --features 500 --steps 5 --warmup 12 > $OUT/goss.log 2>&1 || exit $?
timeout -k 10 400 env LGAP_FSTAMPS=1 python scripts/bench_suite.py --config ltr --rows 2000000 --features 300 --steps 5 --warmup 3 > $OUT/ltr.log 2>&1 || exit $?
grep -E "fstamps|frontier:|^\{" $OUT/goss.log $OUT/ltr.log | cut -c1-260
