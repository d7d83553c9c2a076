# A/B of one LGAP_KERNEL setting against the default at the headline shapes: KNOB=<key=value>
set -u
OUT=gpurun_out/ab_knob
mkdir -p $OUT
for rep in 1 2; do
for v in default "$KNOB"; do
  if [ "$v" = default ]; then unset LGAP_KERNEL; else export LGAP_KERNEL="$v"; fi
  timeout -k 10 200 python3 bench.py --steps 30 --warmup 3 > $OUT/b10.log 2>&1 || exit 1
  timeout -k 10 200 python3 bench.py --rows 1250000 --steps 50 --warmup 5 > $OUT/b1.log 2>&1 || exit 1
  echo "$v 10M $(grep -o '"value": [0-9.]*' $OUT/b10.log) 1.25M $(grep -o '"value": [0-9.]*' $OUT/b1.log)"
done
done
