export TMPDIR=/tmp; mkdir -p gpurun_out
for rows in 10000000 1250000; do
for v in ${VARIANTS:-default pi8 pi32 default}; do
  if [ $v = default ]; then unset LAMBDAGAP_LIB; else export LAMBDAGAP_LIB=$PWD/abvar/lib_$v.so; fi
  timeout -k 10 300 python bench.py --rows $rows --steps 40 --warmup 5 > gpurun_out/ab_${v}_$rows.log 2>&1 || exit $?
  echo $v $rows $(tail -1 gpurun_out/ab_${v}_$rows.log | cut -c100-160)
done; done
