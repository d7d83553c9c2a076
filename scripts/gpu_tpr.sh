#!/bin/bash
# row-per-thread histogram loop (LGAP_HIST_TPR=1): correctness + paired A/B
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
LGAP_HIST_TPR=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "frontier_engine or first_tree or quantized_integer or four_bit" > $OUT/t.log 2>&1; rc=$?
tail -2 $OUT/t.log; [ $rc -ne 0 ] && exit $rc
one() {  # one <label> <env> <args...>
  local lab=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python bench.py "$@" > $OUT/ab.log 2>&1 || exit $?
  echo "$lab: $(grep -E '^\{' $OUT/ab.log | cut -c100-150)"
}
for cfg in "--steps 40 --warmup 3" "--rows 1250000 --steps 40 --warmup 3" "--max-bin 15 --steps 40 --warmup 3" "--quantized --steps 40 --warmup 3"; do
  one "default [$cfg]" X=1 $cfg
  one "tpr     [$cfg]" LGAP_HIST_TPR=1 $cfg
done
