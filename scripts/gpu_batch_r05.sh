#!/bin/bash
# one gpurun call: the partition-tile A/B, then the BASELINE shapes pass
set -u
bash scripts/gpu_ab_r05.sh gpurun_out/ab_part32 "LGAP_KERNEL=part_iters=32" || exit $?
bash scripts/gpu_shapes_r05.sh gpurun_out/shapes
