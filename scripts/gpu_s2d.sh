#!/bin/bash
# binning kernel check + headline kernel trace + secondary configurations (part 1)
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "binning" > $OUT/tb.log 2>&1 || { tail -30 $OUT/tb.log; exit 1; }
tail -1 $OUT/tb.log
timeout -k 10 300 python bench.py --steps 40 --warmup 3 > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
grep -E "^\{" $OUT/bench.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run -- python3 bench.py --steps 10 --warmup 2 > $OUT/prof.log 2>&1 || exit $?
python scripts/prof_summary.py $OUT/prof "10M x 28, 63 leaves (bench.py --steps 10 --warmup 2), session-2 end" 12 > $OUT/prof_summary.md 2>&1
rm -rf $OUT/prof
grep -E "k_pack|k_traverse|k_f_hist|Kernel time" $OUT/prof_summary.md
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -E "^\{" $OUT/$name.log | tail -1 | cut -c1-700
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
run b255 600 python bench.py --num-leaves 255 --steps 500 --warmup 5
run goss12 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 20 --warmup 3
run goss12q 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 20 --warmup 3 --quantized
