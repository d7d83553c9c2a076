#!/bin/bash
# GOSS 12.5M x 500 (fp), session-start library vs current, alternating on one box
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in old new; do
    if [ $lib = old ]; then export LAMBDAGAP_LIB=$PWD/ab_lib/lib_lambdagap_266d1bc.so; else unset LAMBDAGAP_LIB; fi
    timeout -k 10 600 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 20 --warmup 12 > $OUT/g.log 2>&1 || { tail -5 $OUT/g.log; exit 1; }
    echo "$lib $(grep -E '^\{' $OUT/g.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
