#!/bin/bash
# row-per-thread histogram loop (LGAP_FHIST_RPT=1) vs the dword-per-lane loop: frontier
# parity tests under the knob, then alternating paired benches (10M, 1.25M, quantized, 15 bins)
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
true
tail -2 $OUT/rpt_tests.log
b() {  # b <tag> <env> <args...>
  local tag=$1 e=$2; shift 2
  env $e timeout -k 10 300 python bench.py "$@" > $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
  echo "$tag $(grep -E '^\{' $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("auc"))')"
}
for rep in 1 2; do
  b "10M  dw " LGAP_FHIST_RPT=0 --steps 30 --warmup 3
  b "10M  rpt" LGAP_FHIST_RPT=1 --steps 30 --warmup 3
  b "1.25M dw " LGAP_FHIST_RPT=0 --rows 1250000 --steps 50 --warmup 5
  b "1.25M rpt" LGAP_FHIST_RPT=1 --rows 1250000 --steps 50 --warmup 5
done
b "10M q dw " LGAP_FHIST_RPT=0 --quantized --steps 30 --warmup 3
b "10M q rpt" LGAP_FHIST_RPT=1 --quantized --steps 30 --warmup 3
