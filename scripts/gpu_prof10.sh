#!/bin/bash
# frontier tests + 10M / 1.25M / 255-leaf bench lines + rocprofv3 kernel stats at 10M
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
true
true
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -E "^\{" $OUT/$name.log | tail -1 | cut -c1-300
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}



run prof 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof10 -o run -- python3 bench.py --steps 20 --warmup 3
python scripts/prof_summary.py $OUT/prof10 "10M x 28, 63 leaves, frontier engine, frontier r03 v2 (bench.py --steps 20 --warmup 3)" 23 > $OUT/prof10_summary.md 2>&1 || true
head -30 $OUT/prof10_summary.md
LGAP_FSTAMPS=1 run st10 300 python bench.py --steps 3 --warmup 1; grep fstamps $OUT/st10.log
