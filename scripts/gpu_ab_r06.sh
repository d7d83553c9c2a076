#!/bin/bash
# Same-box A/B of two libraries (A = $LIB_A, B = the in-tree build): 10M and 1.25M, alternated.
set -u
OUT=gpurun_out/ab
mkdir -p $OUT
export TMPDIR=/tmp
A=${LIB_A:-variants/lib_r05start.so}
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -n 1 $OUT/$name.log | python3 -c 'import json,sys
try:
    d=json.loads(sys.stdin.read()); print(d["value"])
except Exception: print("?")')"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
# ORDER=ba runs B before A in each pair (checks that the order itself does not bias the pair)
for i in 1 2; do
  if [ "${ORDER:-ab}" = "ba" ]; then
    run B10_$i 300 python bench.py --steps 30 --warmup 5
    run A10_$i 300 env LAMBDAGAP_LIB=$A python bench.py --steps 30 --warmup 5
    run B1_$i 300 python bench.py --rows 1250000 --steps 50 --warmup 5
    run A1_$i 300 env LAMBDAGAP_LIB=$A python bench.py --rows 1250000 --steps 50 --warmup 5
  else
    run A10_$i 300 env LAMBDAGAP_LIB=$A python bench.py --steps 30 --warmup 5
    run B10_$i 300 python bench.py --steps 30 --warmup 5
    run A1_$i 300 env LAMBDAGAP_LIB=$A python bench.py --rows 1250000 --steps 50 --warmup 5
    run B1_$i 300 python bench.py --rows 1250000 --steps 50 --warmup 5
  fi
done
