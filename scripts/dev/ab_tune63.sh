# timed speculation tuner below 128 leaves: default (probing after 64 trees) vs off (LGAP_SPEC_TUNE=0)
set -u
OUT=gpurun_out/ab_tune63
mkdir -p $OUT
for rep in 1 2; do
  for v in off def; do
    if [ $v = off ]; then export LGAP_SPEC_TUNE=0; else unset LGAP_SPEC_TUNE; fi
    timeout -k 10 200 python3 bench.py --steps 500 --warmup 3 > $OUT/l_$v.log 2>&1 || exit 1
    timeout -k 10 200 python3 bench.py > $OUT/d_$v.log 2>&1 || exit 1
    timeout -k 10 200 python3 bench.py --rows 1250000 --steps 500 --warmup 3 > $OUT/s_$v.log 2>&1 || exit 1
    echo "tune=$v 10M/500 $(grep -o '"value": [0-9.]*' $OUT/l_$v.log) default $(grep -o '"value": [0-9.]*' $OUT/d_$v.log) 1.25M/500 $(grep -o '"value": [0-9.]*' $OUT/s_$v.log)"
  done
done
unset LGAP_SPEC_TUNE
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_learner.py -k "speculation or frontier_engine_matches or select_merged" > $OUT/t.log 2>&1 || { tail -20 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
