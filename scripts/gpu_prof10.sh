#!/bin/bash
# frontier tests + 10M / 1.25M / 255-leaf bench lines + rocprofv3 kernel stats at 10M
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "wide_rows or frontier_engine or first_tree or validation_scoring or categorical" > $OUT/t.log 2>&1; rc=$?
tail -3 $OUT/t.log; [ $rc -ne 0 ] && exit $rc
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -E "^\{" $OUT/$name.log | tail -1 | cut -c1-300
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
run b10 300 python bench.py --steps 50 --warmup 3
run b1 300 python bench.py --rows 1250000 --steps 50 --warmup 3
run b255 300 python bench.py --num-leaves 255 --steps 30 --warmup 3
run prof 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof10 -o run -- python3 bench.py --steps 20 --warmup 3
python scripts/prof_summary.py $OUT/prof10 "10M x 28, 63 leaves, frontier engine, 224-block hist (bench.py --steps 20 --warmup 3)" 23 > $OUT/prof10_summary.md 2>&1 || true
head -30 $OUT/prof10_summary.md
