#!/bin/bash
# full GPU suite + smoke, then 512 vs 1024-thread frontier histogram blocks (paired)
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/gputests.log 2>&1 || { tail -30 $OUT/gputests.log; exit 1; }
tail -1 $OUT/gputests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
b() {  # b <tag> <env> <args...>
  local tag=$1 e=$2; shift 2
  env $e timeout -k 10 300 python bench.py "$@" > $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
  echo "$tag $(grep -E '^\{' $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("auc"))')"
}
for rep in 1 2; do
  b "10M  t512 " LGAP_FHIST_THREADS=512 --steps 40 --warmup 3
  b "10M  t1024" LGAP_FHIST_THREADS=1024 --steps 40 --warmup 3
  b "1.25M t512 " LGAP_FHIST_THREADS=512 --rows 1250000 --steps 50 --warmup 5
  b "1.25M t1024" LGAP_FHIST_THREADS=1024 --rows 1250000 --steps 50 --warmup 5
done
b "10M q t512 " LGAP_FHIST_THREADS=512 --quantized --steps 40 --warmup 3
b "10M q t1024" LGAP_FHIST_THREADS=1024 --quantized --steps 40 --warmup 3
