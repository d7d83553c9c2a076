#!/bin/bash
# final secondary lines on the session-2 code
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name	$(grep -E '^\{' $OUT/$name.log | tail -1)"
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
run b10 300 python bench.py --steps 40 --warmup 3
run b10q 300 python bench.py --steps 40 --warmup 3 --quantized
run b1 300 python bench.py --rows 1250000 --steps 50 --warmup 5
run b15 300 python bench.py --max-bin 15 --steps 40 --warmup 3
run ltr 600 python scripts/bench_suite.py --config ltr --rows 5000000 --steps 20 --warmup 5
run ltrq 600 python scripts/bench_suite.py --config ltr --rows 5000000 --steps 20 --warmup 5 --quantized
