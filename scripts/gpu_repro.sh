#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
LGAP_FRONTIER=0 timeout -k 10 300 python scripts/bench_suite.py --config regression_goss --rows 2000000 --features 500 --steps 10 --warmup 12 > $OUT/r2.log 2>&1; rc=$?
echo "seq 2M rc=$rc"; tail -3 $OUT/r2.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
LGAP_FRONTIER=0 timeout -k 10 600 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 10 --warmup 12 > $OUT/r12.log 2>&1; rc=$?
echo "seq 12.5M rc=$rc"; grep -v "^    @" $OUT/r12.log | tail -3 | cut -c1-300
exit $rc
