#!/bin/bash
# frontier histogram grid / chunk size with 1024-thread blocks (10M headline), paired on one box
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
b() {  # b <tag> <env> <args...>
  local tag=$1 e=$2; shift 2
  env $e timeout -k 10 300 python bench.py "$@" > $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
  echo "$tag $(grep -E '^\{' $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
}
for rep in 1 2; do
  b "default(224)   " LGAP_NONE=1 --steps 40 --warmup 3
  b "blocks=256     " LGAP_HIST_BLOCKS=256 --steps 40 --warmup 3
  b "blocks=192     " LGAP_HIST_BLOCKS=192 --steps 40 --warmup 3
  b "min_rows=2048  " LGAP_HIST_MIN_ROWS=2048 --steps 40 --warmup 3
  b "min_rows=512   " LGAP_HIST_MIN_ROWS=512 --steps 40 --warmup 3
done
