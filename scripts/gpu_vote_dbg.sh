#!/bin/bash
# voting over xGMI: which (ranks, top_k) combinations grow the host model (diagnosis runs)
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 LGAP_DP_TRANSPORT=xgmi LGAP_XGMI_TIMEOUT_S=20 DP_LEARNER=voting DP_DIAG=1
for cfg in "3 3" "3 20" "2 3" "4 3" "1 3"; do
  set -- $cfg
  DP_TOPK=$2 timeout -k 10 240 python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nproc-per-node $1 scripts/dp_multirank.py > $OUT/v_$1_$2.log 2>&1
  rc=$?
  echo "ranks $1 topk $2 rc=$rc $(tail -n 1 $OUT/v_$1_$2.log | cut -c1-400)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
