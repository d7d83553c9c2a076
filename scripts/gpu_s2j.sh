#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "quantized or single_rank or multirank_rehearsal" > $OUT/tq.log 2>&1 || { tail -30 $OUT/tq.log; exit 1; }
tail -1 $OUT/tq.log
timeout -k 10 300 python bench.py --steps 40 --warmup 3 --quantized > $OUT/bq.log 2>&1 && grep -E "^\{" $OUT/bq.log | cut -c100-200
LGAP_FRONTIER_STATS=1 timeout -k 10 300 python bench.py --rows 1250000 --steps 40 --warmup 5 --rehearse-dp --quantized > $OUT/bdq.log 2>&1 && grep -E "^\{|frontier:" $OUT/bdq.log | cut -c1-200
