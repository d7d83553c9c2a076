#!/bin/bash
# paired A/B of env settings on the 10M headline (same box): default first, then each setting
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 30 --warmup 3 > $OUT/ab0.log 2>&1 || exit $?
echo "=== default"; grep -E "^\{" $OUT/ab0.log | cut -c1-180
for ab in "$@"; do
  env $ab timeout -k 10 300 python bench.py --steps 30 --warmup 3 > $OUT/ab.log 2>&1 || exit $?
  echo "=== AB $ab"; grep -E "^\{" $OUT/ab.log | cut -c1-180
done
