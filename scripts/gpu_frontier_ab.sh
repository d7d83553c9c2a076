#!/bin/bash
# Frontier engine: kernel trace at 1.25M / 10M rows and a speculation-policy sweep.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
export LGAP_FRONTIER_STATS=1
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -E "frontier:|^\{" $OUT/$name.log | tail -2 | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run check 300 python scripts/frontier_check.py 40000 31 5
for pol in "1 0" "1 8" "0 0" "0 64"; do
  set -- $pol
  LGAP_FRONTIER_POLICY=$1 LGAP_FRONTIER_SPEC=$2 run p$1s$2_1 300 python bench.py --rows 1250000 --steps 30 --warmup 3
  LGAP_FRONTIER_POLICY=$1 LGAP_FRONTIER_SPEC=$2 run p$1s$2_10 300 python bench.py --steps 30 --warmup 3
done
run prof1 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof1 -o run -- python3 bench.py --rows 1250000 --steps 20 --warmup 2
python scripts/prof_summary.py $OUT/prof1 "1.25M rows, frontier" 22 > $OUT/prof1_summary.md
run prof10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof10 -o run -- python3 bench.py --steps 20 --warmup 2
python scripts/prof_summary.py $OUT/prof10 "10M rows, frontier" 22 > $OUT/prof10_summary.md
