#!/bin/bash
# Full GPU validation + headline lines + timeline gaps
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gputests.log 2>&1
rc=$?; echo "gputests rc=$rc"; tail -4 $OUT/gputests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -E "^\{" $OUT/$name.log | tail -1 | cut -c1-200
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
run b10 300 python bench.py --steps 50 --warmup 3
run b1 300 python bench.py --rows 1250000 --steps 50 --warmup 3
run b10q 300 python bench.py --steps 50 --warmup 3 --quantized
run b255 300 python bench.py --num-leaves 255 --steps 30 --warmup 3
timeout -k 10 300 rocprofv3 --kernel-trace -d $PWD/$OUT/ge -o run -- python3 bench.py --steps 20 --warmup 3 > $OUT/ge.log 2>&1 || exit $?
python scripts/prof_gaps.py $OUT/ge 2.0
rm -rf $OUT/ge
