#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/pgf -o run -- python3 scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 10 --warmup 12 > $OUT/pgf.log 2>&1 || exit $?
python scripts/prof_summary.py $OUT/pgf "regression_goss 12.5M x 500, frontier" 22 > $OUT/pgf_summary.md
LGAP_FRONTIER=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/pgs -o run -- python3 scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 10 --warmup 12 > $OUT/pgs.log 2>&1 || exit $?
python scripts/prof_summary.py $OUT/pgs "regression_goss 12.5M x 500, sequential chain" 22 > $OUT/pgs_summary.md
head -22 $OUT/pgf_summary.md; head -22 $OUT/pgs_summary.md
