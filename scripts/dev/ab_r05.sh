# same-box A/B of the round-5 library (variants/lib_r05.so) against the current tree
set -u
OUT=gpurun_out/ab_r05
mkdir -p $OUT
for rep in 1 2; do
for v in cur r05; do
  if [ $v = r05 ]; then export LAMBDAGAP_LIB=$PWD/variants/lib_r05.so; else unset LAMBDAGAP_LIB; fi
  timeout -k 10 200 python3 bench.py --steps 500 --warmup 0 > $OUT/b500_$v.log 2>&1 || exit 1
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $OUT/b20_$v.log 2>&1 || exit 1
  echo "$v 500it $(grep -o '"value": [0-9.]*' $OUT/b500_$v.log) 20st $(grep -o '"value": [0-9.]*' $OUT/b20_$v.log)"
done
done
