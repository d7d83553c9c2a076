#!/bin/bash
# Full GPU validation of the current tree: pytest -m gpu, smoke(), headline bench.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gputests.log 2>&1
rc=$?; echo "gputests rc=$rc"; tail -15 $OUT/gputests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --steps 30 --warmup 3 > $OUT/bench.log 2>&1 || exit $?
tail -1 $OUT/bench.log
for ab in "$@"; do
  env $ab timeout -k 10 300 python bench.py --steps 30 --warmup 3 > $OUT/ab.log 2>&1 || exit $?
  echo "=== AB $ab"; grep -E "^\{" $OUT/ab.log | cut -c1-200
done
