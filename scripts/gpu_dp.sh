#!/bin/bash
# data-parallel paths on the one GPU: single-rank RCCL, multi-rank rehearsals (frontier DP,
# sequential collectives, xGMI), feature / voting parallel
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_learner.py -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -k "data_parallel or feature_parallel or voting" > $OUT/dp.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/dp.log | tail -25; exit $rc
