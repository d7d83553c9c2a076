#!/bin/bash
# select rank sort A/B (+ frontier parity subset), then secondary configurations (part 2)
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_learner.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "frontier or first_tree or forced or auc_parity" > $OUT/tf.log 2>&1 || { tail -30 $OUT/tf.log; exit 1; }
tail -1 $OUT/tf.log
b() {  # b <tag> <env> <args...>
  local tag=$1 e=$2; shift 2
  env $e timeout -k 10 300 python bench.py "$@" > $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
  echo "$tag $(grep -E '^\{' $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("auc"))')"
}
for rep in 1 2; do
  b "10M  rank   " LGAP_NONE=1 --steps 30 --warmup 3
  b "10M  bitonic" LGAP_SEL_BITONIC=1 --steps 30 --warmup 3
  b "1.25M rank   " LGAP_NONE=1 --rows 1250000 --steps 50 --warmup 5
  b "1.25M bitonic" LGAP_SEL_BITONIC=1 --rows 1250000 --steps 50 --warmup 5
done
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -E "^\{" $OUT/$name.log | tail -1 | cut -c1-700
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
run goss12 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 20 --warmup 12
run goss12q 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 20 --warmup 12 --quantized
run vote12 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --learner voting --steps 20 --warmup 12
run ltr 600 python scripts/bench_suite.py --config ltr --rows 5000000 --steps 20 --warmup 5
