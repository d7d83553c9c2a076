set -u
export MASTER_ADDR=127.0.0.1 LGAP_XGMI_TIMEOUT_S=20 DP_LEARNER=voting DP_DIAG=1
run() {
  echo "== $1 topk=$2 world=$3 extra=$4"
  LGAP_DP_TRANSPORT=$1 DP_TOPK=$2 DP_EXTRA="$4" timeout -k 10 150 python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nproc-per-node $3 scripts/dp_multirank.py > gpurun_out/vd_$3_$2.log 2>&1
  echo "exit $?"
  grep -i "fatal\|error\|world\|first differing" gpurun_out/vd_$3_$2.log | grep -v "amdgpu.ids\|hostname\|Gloo" | cut -c1-400 | head -8
  grep -A6 "first differing" gpurun_out/vd_$3_$2.log | head -8
}
run xgmi 2 4 '{"cegb_penalty_split": 0.001}'
run xgmi 20 2 '{"cegb_penalty_split": 0.001, "extra_trees": true}'
run xgmi 2 2 '{"cegb_penalty_split": 0.001, "extra_trees": true}'
