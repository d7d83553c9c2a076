#!/bin/bash
# PMC counter passes of the round-5 headline (three passes, each within the per-block limits:
# 8 SQ + 1 GRBM, FETCH_SIZE + TCC_HIT, WRITE_SIZE + TCC_MISS), summarised per kernel.
set -u
OUT=${1:-gpurun_out/pmc}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $PWD/$OUT/p$i -o run -- python3 bench.py --steps 3 --warmup 1 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python scripts/pmc_summary.py "10M x 28, 63 leaves, round-5 final (bench.py --steps 3 --warmup 1)" $OUT/p1 $OUT/p2 $OUT/p3 > $OUT/pmc_summary.md
rm -rf $OUT/p1 $OUT/p2 $OUT/p3
head -30 $OUT/pmc_summary.md
