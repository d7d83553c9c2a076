#!/bin/bash
# One gpurun pass: GPU test suite, the driver's bench line, the 1.25M (N=8 per-rank share) line,
# and a rocprofv3 kernel-stats profile of the headline. Each step has its own time limit and
# the first failure ends the script. Usage: scripts/gpu_check.sh <outdir> [skip-tests]
set -u
OUT=${1:-gpurun_out/check}
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
  tail -3 $OUT/$name.log | cut -c1-600 >> $OUT/steps.log
  [ $rc -eq 0 ] || exit $rc
}
run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
run bench_1p25 300 python bench.py --rows 1250000 --steps 50 --warmup 5
run prof 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run -- python3 bench.py --steps 20 --warmup 3
python scripts/prof_summary.py $OUT/prof "Headline 10M x 28, 63 leaves" 23 > $OUT/prof_summary.md 2>&1; rm -rf $OUT/prof
if [ "${2:-}" != "skip-tests" ]; then
  run gputests 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
fi
