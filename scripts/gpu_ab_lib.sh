#!/bin/bash
# A/B of library variants (LAMBDAGAP_LIB) on the headline bench, alternating runs.
# usage: gpu_ab_lib.sh <rows> <steps> <variant-name>...   ("default" = lambdagap_amd/lib)
set -o pipefail
mkdir -p gpurun_out
rows=$1; steps=$2; shift 2
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = default ]; then lib=lambdagap_amd/lib/lib_lambdagap.so; else lib=variants/lib_$v.so; fi
    r=$(LAMBDAGAP_LIB=$lib timeout -k 10 180 python -u bench.py --rows $rows --steps $steps --warmup 5 --valid-rows 20000 2>gpurun_out/ab_err.log | tail -1) || exit 1
    echo "$rows $v $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["auc"])')" | tee -a gpurun_out/ab_lib.log
  done
done
