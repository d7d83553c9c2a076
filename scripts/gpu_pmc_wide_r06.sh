#!/bin/bash
# PMC counter passes of the wide shapes: LambdaRank 5M x 300 and GOSS
# regression 12.5M x 500 (255 leaves, bench_suite.py), three passes each within the per-block
# limits, summarised per kernel by scripts/pmc_summary.py.
set -u
OUT=${1:-gpurun_out/pmc_wide}
mkdir -p $OUT
export TMPDIR=/tmp
run_shape() {
  local name=$1; shift
  local i=0
  for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $PWD/$OUT/${name}_p$i -o run -- python3 scripts/bench_suite.py "$@" > $OUT/${name}_p$i.log 2>&1 || { echo "$name pass $i failed"; tail -5 $OUT/${name}_p$i.log; return 1; }
    echo "$name pass $i ok"
  done
  python scripts/pmc_summary.py "$name" $OUT/${name}_p1 $OUT/${name}_p2 $OUT/${name}_p3 > $OUT/${name}_pmc.md
  rm -rf $OUT/${name}_p1 $OUT/${name}_p2 $OUT/${name}_p3
}
SHAPES=${SHAPES:-ltr goss}
for s in $SHAPES; do
  if [ $s = ltr ]; then run_shape ltr5m_x300 --config ltr --rows 5000000 --features 300 --steps 3 --warmup 1 || exit 1; fi
  if [ $s = goss ]; then run_shape goss12m_x500 --config regression_goss --rows 12500000 --features 500 --steps 3 --warmup 11 || exit 1; fi
done
head -20 $OUT/*_pmc.md
