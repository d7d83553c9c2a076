#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_learner.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "objectives or first_tree or auc_parity or metrics or refit or goss" > $OUT/to.log 2>&1 || { tail -30 $OUT/to.log; exit 1; }
tail -1 $OUT/to.log
timeout -k 10 300 python bench.py --steps 40 --warmup 3 > $OUT/b10.log 2>&1 && grep -E "^\{" $OUT/b10.log | cut -c100-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run -- python3 bench.py --steps 10 --warmup 2 > $OUT/prof.log 2>&1 || exit $?
python scripts/prof_summary.py $OUT/prof "10M x 28, 63 leaves" 12 > $OUT/prof_summary.md 2>&1
rm -rf $OUT/prof
grep -E "k_pointwise|Kernel time" $OUT/prof_summary.md
