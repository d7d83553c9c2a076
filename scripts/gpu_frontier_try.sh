#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
export LGAP_FRONTIER_STATS=1
timeout -k 10 300 python scripts/frontier_check.py 40000 31 5 > $OUT/fc1.log 2>&1; rc=$?
echo "fc1 rc=$rc"; tail -5 $OUT/fc1.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --rows 1250000 --steps 30 --warmup 3 > $OUT/fb1.log 2>&1; rc=$?
echo "fb1 rc=$rc"; tail -3 $OUT/fb1.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 3 > $OUT/fb10.log 2>&1; rc=$?
echo "fb10 rc=$rc"; tail -3 $OUT/fb10.log
exit $rc
