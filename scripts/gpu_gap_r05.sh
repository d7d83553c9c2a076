#!/bin/bash
# partition -> histogram boundary: in-kernel stamps with 1024- and 512-thread histogram blocks
set -u
OUT=${1:-gpurun_out/gap}
mkdir -p $OUT
export TMPDIR=/tmp
for th in 1024 512; do
  timeout -k 10 300 env LGAP_FSTAMPS=1 LGAP_KERNEL=fhist_threads=$th python bench.py --steps 10 --warmup 1 > $OUT/st$th.log 2>&1 || exit $?
  echo "=== $th" >> $OUT/steps.log
  grep -E "^\{|fstamps" $OUT/st$th.log | cut -c1-200 >> $OUT/steps.log
done
