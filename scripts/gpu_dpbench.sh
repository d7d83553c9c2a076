#!/bin/bash
# data-parallel frontier on a one-rank RCCL communicator (eager / captured) and a 2-rank host-staged rehearsal
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -E "^\{" $OUT/$name.log | tail -1 | cut -c1-700
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
run dp10 300 python bench.py --rehearse-dp --steps 30 --warmup 3
run dp1 300 python bench.py --rehearse-dp --rows 1250000 --steps 50 --warmup 3
LGAP_DP_GRAPH=1 run dp1g 300 python bench.py --rehearse-dp --rows 1250000 --steps 50 --warmup 3
LGAP_DP_GRAPH=1 run dp10g 300 python bench.py --rehearse-dp --steps 30 --warmup 3
run hs2 600 python bench.py --gpus 2 --dp-host-transport --rows 1250000 --steps 5 --warmup 2
