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
timeout -k 10 300 python bench.py --steps 40 --warmup 3 > $OUT/b10.log 2>&1 && echo "b10 $(grep -E '^\{' $OUT/b10.log | cut -c100-160)"
timeout -k 10 300 python bench.py --rows 1250000 --steps 50 --warmup 5 > $OUT/b1.log 2>&1 && echo "b1 $(grep -E '^\{' $OUT/b1.log | cut -c100-160)"
timeout -k 10 600 python bench.py --num-leaves 255 --steps 500 --warmup 5 > $OUT/b255.log 2>&1 && echo "b255 $(grep -E '^\{' $OUT/b255.log | cut -c100-170)"
