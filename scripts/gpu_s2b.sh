#!/bin/bash
# session 2: full GPU tests after the kernel split, headline bench, DP pipeline A/B,
# row-per-thread histogram A/B
set -u
PROF=0 bash scripts/gpu_check_all.sh && bash scripts/gpu_dp_pipe.sh && bash scripts/gpu_rpt_ab.sh
