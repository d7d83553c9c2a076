#!/bin/bash
# Round-5 phase pass: in-kernel stamps of the frontier rounds (select / scan / hist / partition
# phases) at 10M and 1.25M, and the kernel mix of the owner-computes data-parallel rehearsal
# (one-rank RCCL communicator) at 1.25M. Each step has its own limit; the first failure ends it.
set -u
OUT=${1:-gpurun_out/ph}
mkdir -p $OUT
export TMPDIR=/tmp
( while true; do date > $OUT/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "=== $name" >> $OUT/steps.log
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $OUT/steps.log
  grep -E "^\{|fstamps|frontier:" $OUT/$name.log | cut -c1-400 >> $OUT/steps.log
  [ $rc -eq 0 ] || exit $rc
}
LGAP_FSTAMPS=1 run st10 300 python bench.py --steps 10 --warmup 1
LGAP_FSTAMPS=1 run st1p25 300 python bench.py --rows 1250000 --steps 20 --warmup 3
run pdp 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/pdp -o run -- python3 bench.py --rows 1250000 --steps 20 --warmup 3 --rehearse-dp
python scripts/prof_summary.py $OUT/pdp "owner-computes DP rehearsal, 1.25M x 28, one-rank RCCL" 23 > $OUT/pdp_summary.md 2>&1; rm -rf $OUT/pdp
run p1p25 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/p1 -o run -- python3 bench.py --rows 1250000 --steps 20 --warmup 3
python scripts/prof_summary.py $OUT/p1 "serial frontier, 1.25M x 28" 23 > $OUT/p1_summary.md 2>&1; rm -rf $OUT/p1
