#!/bin/bash
# kernel timeline gaps at 10M and 1.25M (host round trips, launch gaps)
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for rows in 10000000 1250000; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $PWD/$OUT/g$rows -o run -- python3 bench.py --rows $rows --steps 20 --warmup 3 > $OUT/g$rows.log 2>&1 || exit $?
  echo "=== rows $rows"; grep -E "^\{" $OUT/g$rows.log | cut -c1-150
  python scripts/prof_gaps.py $OUT/g$rows 2.0
  rm -rf $OUT/g$rows
done
