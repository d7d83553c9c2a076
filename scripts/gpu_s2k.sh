#!/bin/bash
# PMC counter passes of the headline + a 2-rank self-launched bench.py rehearsal (both ranks
# share the one GPU, host-staged collectives)
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 2 --dp-host-transport --rows 1250000 --steps 5 --warmup 2 > $OUT/r2.log 2>&1; echo "rehearse2 rc=$?"; grep -E '^\{' $OUT/r2.log | cut -c1-400
bash scripts/gpu_round.sh pmc10
