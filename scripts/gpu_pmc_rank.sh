#!/bin/bash
# counters of k_lambdarank (LambdaRank 1M x 300, one pass per counter group)
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD" "SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $pass --kernel-include-regex k_lambdarank --output-format csv -d $PWD/$OUT/pr$i -o run -- python3 scripts/bench_suite.py --config ltr --rows 1000000 --steps 2 --warmup 1 > $OUT/pr$i.log 2>&1 || { echo "pass $i failed"; tail -3 $OUT/pr$i.log; exit 1; }
  f=$(find $OUT/pr$i -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if "lambdarank" not in r.get("Kernel_Name", ""): continue
    acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(acc): print(f"{k:28s} {acc[k]:16.0f}  (records {n[k]})")
PY
done
