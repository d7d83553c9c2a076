#!/bin/bash
# RCCL data-parallel frontier on a one-rank communicator: pipelined exchange vs serial,
# plus a kernel trace of the pipelined run (comm-stream overlap).
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -E "^\{|frontier:" $OUT/$name.log | tail -2 | cut -c1-400
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
export LGAP_FRONTIER_STATS=1
run dp_pipe 300 python bench.py --rows 1250000 --steps 40 --warmup 5 --rehearse-dp
LGAP_DP_PIPELINE=0 run dp_serial 300 python bench.py --rows 1250000 --steps 40 --warmup 5 --rehearse-dp
run dp10_pipe 300 python bench.py --steps 30 --warmup 3 --rehearse-dp
LGAP_DP_PIPELINE=0 run dp10_serial 300 python bench.py --steps 30 --warmup 3 --rehearse-dp
run profdp 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/profdp -o run -- python3 bench.py --rows 1250000 --steps 10 --warmup 2 --rehearse-dp
python scripts/prof_summary.py $OUT/profdp "1.25M rows, RCCL DP frontier (1-rank communicator), pipelined exchange" 12 > $OUT/profdp_summary.md 2>&1
python scripts/prof_overlap.py $OUT/profdp > $OUT/profdp_overlap.md 2>&1 || true; cat $OUT/profdp_overlap.md
rm -rf $OUT/profdp
