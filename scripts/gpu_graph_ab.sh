#!/bin/bash
# graph replay vs eager enqueue of the frontier rounds, 10M and 1.25M; gaps with eager at 10M
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for rows in 10000000 1250000; do
  for g in 1 0 1 0; do
    timeout -k 10 300 python bench.py --rows $rows --graph $g --steps 40 --warmup 3 > $OUT/gab.log 2>&1 || exit $?
    echo "rows $rows graph $g: $(grep -E '^\{' $OUT/gab.log | cut -c100-180)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $PWD/$OUT/ge -o run -- python3 bench.py --graph 0 --steps 20 --warmup 3 > $OUT/ge.log 2>&1 || exit $?
python scripts/prof_gaps.py $OUT/ge 2.0
rm -rf $OUT/ge
