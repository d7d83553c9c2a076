#!/bin/bash
# LambdaRank 5M x 300: kernel time breakdown + frontier stamps; GOSS quantized re-check
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -E "^\{|fstamps|frontier:" $OUT/$name.log | tail -6 | cut -c1-330
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
LGAP_FSTAMPS=1 LGAP_FRONTIER_STATS=1 run ltrst 600 python scripts/bench_suite.py --config ltr --rows 5000000 --steps 3 --warmup 5
run profltr 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/profltr -o run -- python3 scripts/bench_suite.py --config ltr --rows 5000000 --steps 10 --warmup 5
python scripts/prof_summary.py $OUT/profltr "LambdaRank 5M x 300, 255 leaves, frontier engine (bench_suite --steps 10 --warmup 5)" 15 > $OUT/profltr_summary.md 2>&1 || true
head -40 $OUT/profltr_summary.md
run gossq 600 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 20 --warmup 12 --quantized
