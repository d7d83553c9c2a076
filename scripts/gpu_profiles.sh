#!/bin/bash
# kernel traces for profiles/: headline 10M, 1.25M, LambdaRank 5M x 300, GOSS 12.5M x 500 (quantized), stamps at 10M
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
prof() {  # prof <name> <title> <iters> <cmd...>
  local name=$1 title=$2 iters=$3; shift 3
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/$name -o run -- "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -E "^\{" $OUT/$name.log | tail -1 | cut -c1-200
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
  python scripts/prof_summary.py $OUT/$name "$title" $iters > $OUT/${name}_summary.md 2>&1 || true
  rm -rf $OUT/$name
}
prof p10 "10M x 28, 63 leaves, frontier engine, round 3 (bench.py --steps 20 --warmup 3)" 23 python3 bench.py --steps 20 --warmup 3
prof p1 "1.25M x 28 (per-rank share at N=8), 63 leaves, frontier engine, round 3 (bench.py --rows 1250000 --steps 40 --warmup 3)" 43 python3 bench.py --rows 1250000 --steps 40 --warmup 3
prof pq "10M x 28, 63 leaves, use_quantized_grad (int8-level histograms), round 3" 23 python3 bench.py --steps 20 --warmup 3 --quantized
prof pltr "LambdaRank 5M x 300, 255 leaves, frontier engine, 150 KB LDS tiles, round 3 (bench_suite --steps 10 --warmup 5)" 15 python3 scripts/bench_suite.py --config ltr --rows 5000000 --steps 10 --warmup 5
prof pgoss "regression EFB+GOSS 12.5M x 500, 255 leaves, quantized, round 3 (bench_suite --steps 10 --warmup 12)" 22 python3 scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 10 --warmup 12 --quantized
LGAP_FSTAMPS=1 timeout -k 10 300 python bench.py --steps 10 --warmup 1 > $OUT/st10.log 2>&1 || exit $?
grep -E "fstamps|frontier:" $OUT/st10.log
