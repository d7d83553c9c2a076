#!/bin/bash
# session 2 (continued): remaining GPU tests, headline bench, DP pipeline A/B, row-per-thread A/B
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_learner.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "row_per_thread or wide_rows or cegb or pool_bound or data_parallel_path" > $OUT/t2.log 2>&1 || { tail -30 $OUT/t2.log; exit 1; }
tail -2 $OUT/t2.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash scripts/gpu_dp_pipe.sh && bash scripts/gpu_rpt_ab.sh
