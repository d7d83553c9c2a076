#!/bin/bash
# Frontier diagnostics: in-kernel phase stamps (1.25M / 10M) and PMC passes at 10M.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc"; grep -E "fstamps|^\{" $OUT/$name.log | cut -c1-220
  if [ $rc -ne 0 ]; then exit $rc; fi
}
LGAP_FSTAMPS=1 run st1 300 python bench.py --rows 1250000 --steps 3 --warmup 1
LGAP_FSTAMPS=1 run st10 300 python bench.py --steps 3 --warmup 1
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum"; do
  n=$(echo $pass | cut -c1-8 | tr -d ' ')
  run pmc_$n 240 timeout -s KILL 200 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $PWD/$OUT/pmcf_$n -o run -- python3 bench.py --steps 3 --warmup 1
done
python scripts/pmc_summary.py "10M x 28, 63 leaves, frontier engine (bench.py --steps 3 --warmup 1)" $OUT/pmcf_* > $OUT/pmcf_summary.md
cat $OUT/pmcf_summary.md
