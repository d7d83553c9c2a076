#!/bin/bash
# GPU tests, then score-update A/B (leaf ranges vs LDS-staged traversal) at 10M and 1.25M rows.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -p no:cacheprovider > gpurun_out/gput.log 2>&1; rc=$?; echo gpu tests rc=$rc; tail -2 gpurun_out/gput.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for p in leaves traverse; do
  LGAP_SCORE_PATH=$p timeout -k 10 300 python bench.py --steps 30 --warmup 3 > gpurun_out/b10_$p.log 2>&1 || exit $?
  echo $p 10M; tail -1 gpurun_out/b10_$p.log | cut -c100-200
  LGAP_SCORE_PATH=$p timeout -k 10 300 python bench.py --rows 1250000 --steps 50 --warmup 5 > gpurun_out/b1_$p.log 2>&1 || exit $?
  echo $p 1.25M; tail -1 gpurun_out/b1_$p.log | cut -c100-200
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 2 > gpurun_out/prof.log 2>&1 || exit $?
python scripts/prof_summary.py gpurun_out/prof "10M rows x 28, 63 leaves" 22 > gpurun_out/prof_summary.md
