#!/bin/bash
# Frontier iteration check: parity vs sequential/CPU, stamps, benches (+ optional A/B env pairs).
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
export LGAP_FRONTIER_STATS=1
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -E "fstamps|frontier:|^\{" $OUT/$name.log | tail -7 | cut -c1-240
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run check 300 python scripts/frontier_check.py 40000 31 5
LGAP_FSTAMPS=1 run st10 300 python bench.py --steps 3 --warmup 1
run b1 300 python bench.py --rows 1250000 --steps 30 --warmup 3
run b10 300 python bench.py --steps 30 --warmup 3
for ab in "$@"; do
  env $ab timeout -k 10 300 python bench.py --steps 30 --warmup 3 > $OUT/ab.log 2>&1 || exit $?
  echo "=== AB $ab"; grep -E "^\{" $OUT/ab.log | cut -c1-200
done
