#!/bin/bash
# Round-5 final pass, part 1: full GPU suite, smoke, the driver's bench line, a rocprofv3 kernel
# profile and in-kernel stamps of the headline, the 1.25M / 1M lines, the owner-computes rehearsal.
set -u
OUT=${1:-gpurun_out/final2}
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
  grep -E "^\{|passed|failed|fstamps|frontier:|smoke ok" $OUT/$name.log | cut -c1-330 >> $OUT/steps.log
  [ $rc -eq 0 ] || exit $rc
}
run gputests 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
run bench40 300 python bench.py --steps 40 --warmup 5
run b1p25 300 python bench.py --rows 1250000 --steps 50 --warmup 5
run b1m 300 python bench.py --rows 1000000 --steps 50 --warmup 5
run owner1p25 300 python bench.py --rows 1250000 --steps 50 --warmup 5 --rehearse-dp
run st10 300 env LGAP_FSTAMPS=1 python bench.py --steps 10 --warmup 1
run prof 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run -- python3 bench.py --steps 20 --warmup 3
python scripts/prof_summary.py $OUT/prof "Headline 10M x 28, 63 leaves (round-5 final)" 23 > $OUT/prof_summary.md 2>&1; rm -rf $OUT/prof
