#!/bin/bash
# Same-box kernel tables of two libraries (A = $LIB_A, B = in-tree) at 10M x 28, 63 leaves.
set -u
OUT=gpurun_out/abprof
mkdir -p $OUT
export TMPDIR=/tmp
A=${LIB_A:-variants/lib_r05start.so}
LAMBDAGAP_LIB=$A timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/A -o run -- python3 bench.py --steps 20 --warmup 2 > $OUT/A.log 2>&1 || exit $?
python scripts/prof_summary.py $OUT/A "A: round-start library, 10M" 22 > $OUT/A_summary.md
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/B -o run -- python3 bench.py --steps 20 --warmup 2 > $OUT/B.log 2>&1 || exit $?
python scripts/prof_summary.py $OUT/B "B: current library, 10M" 22 > $OUT/B_summary.md
