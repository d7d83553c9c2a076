#!/bin/bash
# Quick GPU validation + timing of the current tree: learner/kernel tests, phase stamps,
# 1.25M and 10M benches. Stops at the first failing step.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_learner.py -p no:cacheprovider > $OUT/gpul.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/gpul.log
[ $rc -ne 0 ] && exit $rc
LGAP_STAMPS=1 timeout -k 10 300 python bench.py --rows 1250000 --steps 2 --warmup 1 > $OUT/stampsmall.log 2>&1 || exit $?
grep stamps $OUT/stampsmall.log
timeout -k 10 300 python bench.py --rows 1250000 --steps 50 --warmup 5 > $OUT/small.log 2>&1 || exit $?
tail -1 $OUT/small.log
timeout -k 10 300 python bench.py --steps 30 --warmup 3 > $OUT/bench.log 2>&1 || exit $?
tail -1 $OUT/bench.log
