#!/bin/bash
# A/B of the k_reduce_scan fold shape (compile-time LGAP_SCAN_FOLD) via LAMBDAGAP_LIB
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_scanfold.log
for rows in 10000000 1250000; do
  for v in default f2 default f2; do
    if [ $v = default ]; then lib=lambdagap_amd/lib/lib_lambdagap.so; else lib=ab_variants/lib_$v.so; fi
    r=$(LAMBDAGAP_LIB=$lib timeout -k 10 120 python -u bench.py --rows $rows --steps 40 --warmup 5 --valid-rows 20000 2>gpurun_out/ab_err.log | tail -1) || exit 1
    echo "$rows $v $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["auc"])')" | tee -a gpurun_out/ab_scanfold.log
  done
done
echo "=== gpu tests on the f2 variant"
LAMBDAGAP_LIB=ab_variants/lib_f2.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_f2.log 2>&1 || { tail -30 gpurun_out/gputests_f2.log; exit 1; }
tail -2 gpurun_out/gputests_f2.log
