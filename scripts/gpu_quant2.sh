#!/bin/bash
# quantized hist MODE 3 (32-bit LDS bins) vs MODE 2 (64-bit LDS bins)
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "quantized" > $OUT/t.log 2>&1; rc=$?
tail -3 $OUT/t.log; [ $rc -ne 0 ] && exit $rc
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -E "^\{" $OUT/$name.log | tail -1 | cut -c1-330
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
run b10q 300 python bench.py --steps 50 --warmup 3 --quantized
LGAP_QUANT_LDS32=0 run b10q64 300 python bench.py --steps 50 --warmup 3 --quantized
run ltrq 600 python scripts/bench_suite.py --config ltr --rows 5000000 --steps 20 --warmup 5 --quantized
LGAP_QUANT_LDS32=0 run ltrq64 600 python scripts/bench_suite.py --config ltr --rows 5000000 --steps 20 --warmup 5 --quantized
run gossq 600 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 20 --warmup 12 --quantized
