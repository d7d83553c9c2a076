#!/bin/bash
set -u
bash scripts/gpu_gap_r05.sh gpurun_out/gap || exit $?
bash scripts/gpu_final3_r05.sh gpurun_out/final3
