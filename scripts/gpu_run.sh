#!/bin/bash
# One gpurun call, parameterised: each named step runs under its own time limit and the call
# stops at the first failing step (no GPU work after a fault, abort or time-out).
#   bash scripts/gpu_run.sh tests:<pytest files>[|<-k expression>] | smoke | bench:<bench args> | prof:<bench args> | py:<script args> | sh:<command> ...
# e.g. bash scripts/gpu_run.sh "tests:tests/test_device_metrics.py" "bench:--steps 40 --warmup 3"
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for step in "$@"; do
  i=$((i + 1))
  kind=${step%%:*}
  arg=${step#*:}
  [ "$arg" = "$step" ] && arg=""
  log=$OUT/step${i}_${kind}.log
  case $kind in
    tests) files=${arg%%|*}; kexpr=""; [ "$files" != "$arg" ] && kexpr=${arg#*|}
           if [ -n "$kexpr" ]; then
             timeout -k 10 900 python -u -m pytest ${files:-tests -m gpu} -k "$kexpr" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $log 2>&1
           else
             timeout -k 10 900 python -u -m pytest ${files:-tests -m gpu} -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $log 2>&1
           fi ;;
    smoke) timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $log 2>&1 ;;
    bench) timeout -k 10 400 python bench.py $arg > $log 2>&1 ;;
    prof)  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof$i -o run -- python3 bench.py $arg > $log 2>&1 &&
             python scripts/prof_summary.py $OUT/prof$i "bench.py $arg" 12 > $OUT/prof${i}_summary.md 2>&1 && rm -rf $OUT/prof$i ;;
    py)    timeout -k 10 600 python -u $arg > $log 2>&1 ;;
    sh)    timeout -k 10 600 bash -c "$arg" > $log 2>&1 ;;
    # three counter passes (one per block budget: SQ / TCC fetch / TCC write), each in its own
    # run, summarised per kernel by scripts/pmc_summary.py; <args>: a python script and its
    # arguments (e.g. pmc:bench.py --steps 3 --warmup 1)
    pmc)   rc=0; j=0
           for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum"; do
             j=$((j + 1))
             timeout -s KILL 240 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $PWD/$OUT/pmc${i}_$j -o run -- python3 $arg >> $log 2>&1 || { rc=$?; break; }
           done
           if [ $rc -eq 0 ]; then
             python scripts/pmc_summary.py "$arg" $OUT/pmc${i}_* > $OUT/pmc${i}_summary.md 2>&1; rm -rf $OUT/pmc${i}_[0-9]
             head -20 $OUT/pmc${i}_summary.md
           fi
           (exit $rc) ;;
    # one counter pass of your own: pmcx:<counters>|<python script and args>; the per-kernel means
    # of each counter land in pmcx<i>_summary.csv
    pmcx)  ctrs=${arg%%|*}; prog=${arg#*|}
           timeout -s KILL 240 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $PWD/$OUT/pmcx$i -o run -- python3 $prog > $log 2>&1 &&
             python scripts/pmc_counters.py $OUT/pmcx$i > $OUT/pmcx${i}_summary.csv 2>&1 && rm -rf $OUT/pmcx$i && head -20 $OUT/pmcx${i}_summary.csv ;;
    *) echo "unknown step $kind"; exit 2 ;;
  esac
  rc=$?
  echo "=== step $i $kind rc=$rc"; tail -4 $log | cut -c1-400
  [ -f $OUT/prof${i}_summary.md ] && head -24 $OUT/prof${i}_summary.md
  if [ $rc -ne 0 ]; then exit $rc; fi
done
