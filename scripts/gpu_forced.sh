#!/bin/bash
# forced splits on the frontier + lambdarank discount table + frontier regression tests
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_learner.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "forced or frontier_engine or first_tree or lambdarank or quantized or position or four_bit or wide_rows" > $OUT/t.log 2>&1; rc=$?
tail -15 $OUT/t.log; [ $rc -ne 0 ] && exit $rc
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -E "^\{" $OUT/$name.log | tail -1 | cut -c1-250
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
run b10 300 python bench.py --steps 40 --warmup 3
run ltr 600 python scripts/bench_suite.py --config ltr --rows 5000000 --steps 20 --warmup 5
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/pl -o run -- python3 scripts/bench_suite.py --config ltr --rows 5000000 --steps 5 --warmup 2 > $OUT/pl.log 2>&1 || exit $?
python scripts/prof_summary.py $OUT/pl "LambdaRank 5M x 300 (LDS discount table)" 7 > $OUT/pl_summary.md 2>&1; grep -E "k_lambdarank|k_f_hist" $OUT/pl_summary.md
rm -rf $OUT/pl
run b15 300 python bench.py --max-bin 15 --steps 40 --warmup 3
LGAP_NIBBLE=0 run b15n 300 python bench.py --max-bin 15 --steps 40 --warmup 3
