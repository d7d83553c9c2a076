#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_learner.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "frontier or forced or cegb or first_tree or single_rank" > $OUT/tf.log 2>&1 || { tail -30 $OUT/tf.log; exit 1; }
tail -1 $OUT/tf.log
timeout -k 10 300 python bench.py --steps 40 --warmup 3 > $OUT/b.log 2>&1 && grep -o "\"value\": [0-9.]*" $OUT/b.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run -- python3 bench.py --steps 10 --warmup 2 > $OUT/prof.log 2>&1 || exit $?
python scripts/prof_summary.py $OUT/prof "10M x 28, 63 leaves (bench.py --steps 10 --warmup 2), session-2 final" 12 > $OUT/prof_summary.md 2>&1
rm -rf $OUT/prof
grep -E "k_f_results|k_f_select|Kernel time" $OUT/prof_summary.md
