#!/bin/bash
# GPU check sequence for one gpurun call. Every GPU step has its own time limit;
# the script stops at the first fault / abort / timeout (anything other than a
# clean exit or an ordinary pytest failure).
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <limit-seconds> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "=== $name" | tee -a $OUT/steps.log
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -5 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    info) step info 300 python -c "import lambdagap_amd as l; print('devices', l.device_count())";;
    kernels) step kernels 900 python -m pytest tests/test_gpu_kernels.py -q --timeout 300 -p no:cacheprovider;;
    dp1) step dp1 600 python -u -m pytest tests/test_gpu_learner.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "single_rank";;
    xg) step xg 1000 python -u -m pytest tests/test_gpu_learner.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "xgmi or single_rank";;
    xgbench) step x1single 300 python bench.py --rows 1250000 --steps 50 --warmup 5 && LGAP_DP_TRANSPORT=xgmi step x1xgmi 300 python bench.py --rows 1250000 --steps 50 --warmup 5 --rehearse-dp && LGAP_DP_TRANSPORT=collective step x1coll 300 python bench.py --rows 1250000 --steps 50 --warmup 5 --rehearse-dp && step x10single 300 python bench.py --steps 30 --warmup 3 && LGAP_DP_TRANSPORT=xgmi step x10xgmi 300 python bench.py --steps 30 --warmup 3 --rehearse-dp;;
    xgq) LGAP_DP_TRANSPORT=xgmi step x1xgmi 300 python bench.py --rows 1250000 --steps 50 --warmup 5 --rehearse-dp && LGAP_DP_TRANSPORT=xgmi step x10xgmi 300 python bench.py --steps 30 --warmup 3 --rehearse-dp && step x1single 300 python bench.py --rows 1250000 --steps 50 --warmup 5;;
    xgprof) LGAP_DP_TRANSPORT=xgmi step xgprof 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/xgprof -o run -- python3 bench.py --rows 1250000 --steps 20 --warmup 2 --rehearse-dp && python scripts/prof_summary.py $OUT/xgprof "1.25M rows, DP frontier xGMI (1 rank)" 22 > $OUT/xgprof_summary.md;;
    learnerv) step learnerv 900 python -u -m pytest tests/test_gpu_learner.py tests/test_frontier_kernels.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider;;
    shapes) step goss3m 600 python scripts/bench_suite.py --config regression_goss --rows 3000000 --features 500 --steps 10 --warmup 2 && step ltr2m 600 python scripts/bench_suite.py --config ltr --rows 2000000 --features 300 --steps 10 --warmup 2;;
    xgstamps) LGAP_FSTAMPS=1 LGAP_DP_TRANSPORT=xgmi step xgstamps 300 python bench.py --rows 1250000 --steps 12 --warmup 2 --rehearse-dp && LGAP_FSTAMPS=1 step serstamps 300 python bench.py --rows 1250000 --steps 12 --warmup 2 && LGAP_FSTAMPS=1 LGAP_DP_TRANSPORT=xgmi step xgstamps10 300 python bench.py --steps 12 --warmup 2 --rehearse-dp;;
    mono) step mono 900 python scripts/bench_monotone.py --rows 1000000 --steps 20 --warmup 3;;
    rehearse2x) step rehearse2x 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dp-host-transport --rows 1250000 --steps 20 --warmup 3;;
    monotag) LGAP_TIMETAG=1 step monotag 300 python scripts/bench_monotone.py --rows 1000000 --steps 10 --warmup 2 --methods intermediate;;
    big100) step big100 1150 python -u scripts/big_stream.py --rows 100000000 --features 500 --chunk 2000000 --steps 5 --warmup 1;;
    big25) step big25 900 python -u scripts/big_stream.py --rows 25000000 --features 500 --chunk 2000000 --steps 5 --warmup 1;;
    vote12) step vote12 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --learner voting --steps 10 --warmup 3;;
    voteprof) step voteprof 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/voteprof -o run -- python3 scripts/bench_suite.py --config regression_goss --rows 3000000 --features 500 --learner voting --steps 10 --warmup 2 && python scripts/prof_summary.py $OUT/voteprof "GOSS 3M x 500 voting, one rank" 12 > $OUT/voteprof_summary.md && step serprof3 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/serprof3 -o run -- python3 scripts/bench_suite.py --config regression_goss --rows 3000000 --features 500 --steps 10 --warmup 2 && python scripts/prof_summary.py $OUT/serprof3 "GOSS 3M x 500 serial" 12 > $OUT/serprof3_summary.md;;
    votet) step votet 600 python -u -m pytest tests/test_gpu_learner.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "voting";;
    vote3) step vote3 600 python scripts/bench_suite.py --config regression_goss --rows 3000000 --features 500 --learner voting --steps 10 --warmup 2 && step ser3 600 python scripts/bench_suite.py --config regression_goss --rows 3000000 --features 500 --steps 10 --warmup 2;;
    bagt) step bagt 600 python -u -m pytest tests/test_gpu_learner.py tests/test_gpu_kernels.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "bag or goss";;
    gossprof) step gossprof 900 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/gossprof -o run -- python3 scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 5 --warmup 11 && python scripts/prof_summary.py $OUT/gossprof "GOSS 12.5M x 500 serial, bagged iterations" 16 > $OUT/gossprof_summary.md;;
    oobab) for r in 2 4 8; do LGAP_KERNEL=oob_rows=$r step oob$r 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/oob$r -o run -- python3 scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 4 --warmup 11 && python scripts/prof_summary.py $OUT/oob$r "GOSS 12.5M x 500, oob_rows=$r" 15 > $OUT/oob${r}_summary.md || exit 1; done;;
    ict) step ict 600 python -u -m pytest tests/test_gpu_learner.py tests/test_frontier_kernels.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "interaction or frontier or bynode";;
    dpmulti) step dpmulti 1100 python -u -m pytest tests/test_gpu_learner.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "multirank";;
    fp) step fp 600 python -u -m pytest tests/test_gpu_learner.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "feature_parallel";;
    dpbench) step b1single 300 python bench.py --rows 1250000 --steps 50 --warmup 5 && LGAP_DP_TRANSPORT=xgmi step b1xgmi 300 python bench.py --rows 1250000 --steps 50 --warmup 5 --rehearse-dp && LGAP_DP_TRANSPORT=collective step b1coll 300 python bench.py --rows 1250000 --steps 50 --warmup 5 --rehearse-dp && step b10single 300 python bench.py --steps 30 --warmup 3 && LGAP_DP_TRANSPORT=xgmi step b10xgmi 300 python bench.py --steps 30 --warmup 3 --rehearse-dp;;
    profdpx) LGAP_DP_TRANSPORT=xgmi step profdpx 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/profdpx -o run -- python3 bench.py --rows 1250000 --steps 20 --warmup 2 --rehearse-dp && python scripts/prof_summary.py $OUT/profdpx "1.25M rows, DP xGMI path (1 rank)" 22 > $OUT/profdpx_summary.md;;
    pmc10) for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum"; do
             n=$(echo $pass | cut -c1-8 | tr -d ' '); step pmc_$n 240 timeout -s KILL 200 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $PWD/$OUT/pmc10_$n -o run -- python3 bench.py --steps 3 --warmup 1;
           done; python scripts/pmc_summary.py "10M x 28, 63 leaves (bench.py --steps 3 --warmup 1)" $OUT/pmc10_* > $OUT/pmc10_summary.md;;
    stampsdp) LGAP_STAMPS=1 LGAP_DP_TRANSPORT=xgmi step stampsdp 300 python bench.py --rows 1250000 --steps 3 --warmup 1 --rehearse-dp;;
    quick) step b10 300 python bench.py --steps 30 --warmup 3 && step b1 300 python bench.py --rows 1250000 --steps 50 --warmup 5;;
    diagrank) step diagrank 300 python scripts/diag_rank.py ${DIAG_TARGET:-lambdagap-s} && step diagrank_dp 300 python scripts/diag_rank.py ${DIAG_TARGET:-lambdagap-s} gpu_use_dp=true;;
    dpfix) step dpfix 900 python -u -m pytest tests/test_gpu_learner.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "multirank or watchdog or xgmi_exchange";;
    vote) step vote 900 python -u -m pytest tests/test_gpu_learner.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "voting or multirank";;
    evidence) step parity1m 600 python -u -m pytest tests/test_gpu_learner.py -x -v --timeout 500 --timeout-method thread -p no:cacheprovider -k "fixed_point_vs_fp64" && step b255 600 python bench.py --num-leaves 255 --steps 500 --warmup 5 && step b63dp 600 python bench.py --use-dp --steps 30 --warmup 3 && step vote12 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --learner voting --steps 20 --warmup 3 && step serial12 900 python scripts/bench_suite.py --config regression_goss --rows 12500000 --features 500 --steps 20 --warmup 3 && step parity10 1000 python scripts/auc_parity.py --rows 10000000 --iters 50;;
    abchunks) step c10a 300 python bench.py --steps 30 --warmup 3 && LGAP_SCAN_CHUNKS=1 step c10b 300 python bench.py --steps 30 --warmup 3 && step c1a 300 python bench.py --rows 1250000 --steps 50 --warmup 5 && LGAP_SCAN_CHUNKS=1 step c1b 300 python bench.py --rows 1250000 --steps 50 --warmup 5 && LGAP_SCAN_CHUNKS=4 step c10c 300 python bench.py --steps 30 --warmup 3;;
    rehearse2) step rehearse2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dp-host-transport --rows 1250000 --steps 5 --warmup 2;;
    learnerx) step learnerx 400 python -m pytest tests/test_gpu_learner.py -x -q --timeout 60 -p no:cacheprovider;;
    learner) step learner 1200 python -m pytest tests/test_gpu_learner.py -q --timeout 300 -p no:cacheprovider;;
    gputests) step gputests 1500 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()";;
    bench1m) step bench1m 400 python bench.py --rows 1000000 --steps 10 --warmup 2;;
    bench) step bench 900 python bench.py --steps 30 --warmup 3;;
    benchdp) step benchdp 900 python bench.py --steps 30 --warmup 3 --rehearse-dp;;
    abpost) step abpost10 900 python scripts/ab_bench.py --rows 10000000 --variant device_post_mode=1 --variant device_post_mode=2 --variant device_post_mode=0 && step abpost1 900 python scripts/ab_bench.py --rows 1250000 --variant device_post_mode=1 --variant device_post_mode=2 --variant device_post_mode=0;;
    abfused) step abfused10 900 python scripts/ab_bench.py --rows 10000000 --variant device_fused_partition=1 --variant device_fused_partition=0 && step abfused1 900 python scripts/ab_bench.py --rows 1250000 --variant device_fused_partition=1 --variant device_fused_partition=0;;
    abhist) step abhist10 900 python scripts/ab_bench.py --rows 10000000 --variant device_fused_hist=1 --variant device_fused_hist=0 && step abhist1 900 python scripts/ab_bench.py --rows 1250000 --variant device_fused_hist=1 --variant device_fused_hist=0;;
    abminrows) step abmr10 900 python scripts/ab_bench.py --rows 10000000 --variant device_hist_min_rows=2048 --variant device_hist_min_rows=1024 --variant device_hist_min_rows=512 --variant device_hist_min_rows=4096 && step abmr1 900 python scripts/ab_bench.py --rows 1250000 --variant device_hist_min_rows=2048 --variant device_hist_min_rows=1024 --variant device_hist_min_rows=512;;
    abgraph) step ab10 900 python scripts/ab_bench.py --rows 10000000 && step ab1 900 python scripts/ab_bench.py --rows 1250000;;
    quad) step q10g 600 python bench.py --steps 30 --warmup 3 --graph 1 && step q10e 600 python bench.py --steps 30 --warmup 3 --graph 0 && step q1g 600 python bench.py --rows 1250000 --steps 50 --warmup 5 --graph 1 && step q1e 600 python bench.py --rows 1250000 --steps 50 --warmup 5 --graph 0;;
    nograph) step nograph 600 python bench.py --steps 30 --warmup 3 --graph 0 && step nographsmall 600 python bench.py --rows 1250000 --steps 50 --warmup 5 --graph 0;;
    dpself) step dpself 600 python scripts/dp_selftest.py;;
    small) step small 600 python bench.py --rows 1250000 --steps 50 --warmup 5 && step smalldp 600 python bench.py --rows 1250000 --steps 50 --warmup 5 --rehearse-dp;;
    timetag) LGAP_TIMETAG=1 step timetag 900 python bench.py --steps 20 --warmup 3;;
    pmc) step pmc 900 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA --kernel-trace --output-format csv -d $PWD/$OUT/pmc -o pmc -- python3 bench.py --rows 2000000 --steps 3 --warmup 1;;
    profpost) LGAP_SPLIT_POST=1 step profpost 900 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/profpost -o run -- python3 bench.py --steps 10 --warmup 2;;
    stamps) LGAP_STAMPS=1 step stamps 600 python bench.py --rows 10000000 --steps 2 --warmup 1;;
    stampsmall) LGAP_STAMPS=1 step stampsmall 600 python bench.py --rows 1250000 --steps 2 --warmup 1;;
    profsmall) step profsmall 900 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/profsmall -o run -- python3 bench.py --rows 1250000 --steps 20 --warmup 2 && python scripts/prof_summary.py $OUT/profsmall "1.25M rows, graph path" 22 > $OUT/profsmall_summary.md;;
    profsmalldp) step profsmalldp 900 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/profsmalldp -o run -- python3 bench.py --rows 1250000 --steps 20 --warmup 2 --rehearse-dp && python scripts/prof_summary.py $OUT/profsmalldp "1.25M rows, DP rehearsal path" 22 > $OUT/profsmalldp_summary.md;;
    marker) step marker 900 rocprofv3 --marker-trace --kernel-trace --stats -d $PWD/$OUT/marker -o run -- python3 bench.py --rows 1250000 --steps 10 --warmup 2 --rehearse-dp;;
    watchdog) step watchdog 300 python scripts/watchdog_selftest.py;;
    prof) step prof 900 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run -- python3 bench.py --steps 20 --warmup 2 && python scripts/prof_summary.py $OUT/prof "10M rows x 28, 63 leaves" 22 > $OUT/prof_summary.md;;
  esac
done
echo ALLDONE
