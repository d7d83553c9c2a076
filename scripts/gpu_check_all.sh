#!/bin/bash
# One gpurun call: the driver's round-end tiers (pytest -m gpu, smoke, bench) plus a
# kernel-trace profile of the headline. Stops at the first failing GPU step.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; tail -3 $OUT/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run gputests 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
run bench 300 python bench.py --steps 40 --warmup 3
if [ "${PROF:-1}" = 1 ]; then
  run prof 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run -- python3 bench.py --steps 10 --warmup 2
  python scripts/prof_summary.py $OUT/prof "10M x 28, 63 leaves (bench.py --steps 10 --warmup 2)" 12 > $OUT/prof_summary.md 2>&1
  rm -rf $OUT/prof
  head -30 $OUT/prof_summary.md
fi
