# multi-rank rehearsals at 255 leaves (the select's merged alive order on the distributed paths)
set -u
export MASTER_ADDR=127.0.0.1 LGAP_XGMI_TIMEOUT_S=30 DP_ROWS=200000
for L in data voting feature; do
  DP_LEARNER=$L LGAP_DP_TRANSPORT=xgmi DP_EXTRA='{"num_leaves": 255, "min_data_in_leaf": 5}' timeout -k 10 200 python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nproc-per-node 2 scripts/dp_multirank.py > gpurun_out/dp255_$L.log 2>&1
  echo "$L exit $? $(grep -o '"ranks_identical": [a-z]*\|"identical_leading_trees": [0-9]*\|"max_abs_diff_vs_cpu_dp": [0-9.e-]*' gpurun_out/dp255_$L.log | tr '\n' ' ')"
done
