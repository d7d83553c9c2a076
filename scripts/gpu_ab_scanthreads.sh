#!/bin/bash
# A/B of the k_reduce_scan block size (compile-time LGAP_SCAN_THREADS) via LAMBDAGAP_LIB
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_scanthreads.log
for rows in 10000000 1250000; do
  for v in default t512 t256 default t512 t256; do
    if [ $v = default ]; then lib=lambdagap_amd/lib/lib_lambdagap.so; else lib=ab_variants/lib_$v.so; fi
    r=$(LAMBDAGAP_LIB=$lib timeout -k 10 120 python -u bench.py --rows $rows --steps 40 --warmup 5 --valid-rows 20000 2>gpurun_out/ab_err.log | tail -1) || exit 1
    echo "$rows $v $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["auc"])')" | tee -a gpurun_out/ab_scanthreads.log
  done
done
