#!/bin/bash
# DP graph capture check: GPU tests, then the 1.25M DP rehearsal with and without capture.
set -o pipefail
mkdir -p gpurun_out
echo "=== gputests"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?; echo "gputests rc=$rc"; tail -3 gpurun_out/gputests.log; [ $rc -eq 0 ] || exit $rc
for g in 1 0; do
  echo "=== dp rehearsal LGAP_DP_GRAPH=$g"
  LGAP_DP_GRAPH=$g timeout -k 10 180 python -u bench.py --rows 1250000 --rehearse-dp --steps 60 --warmup 5 > gpurun_out/dpg$g.log 2>&1
  rc=$?; tail -1 gpurun_out/dpg$g.log; [ $rc -eq 0 ] || exit $rc
done
echo "=== headline"
timeout -k 10 240 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
echo ALLDONE
