#!/bin/bash
set -u
mkdir -p gpurun_out/cl
timeout -k 10 300 python -u -m pytest tests/test_gpu_learner.py -x -v --timeout 250 --timeout-method thread -k "concurrent_gpu_load" > gpurun_out/cl/test.log 2>&1 || { tail -30 gpurun_out/cl/test.log; exit 1; }
tail -3 gpurun_out/cl/test.log
bash scripts/gpu_pmc_r05.sh gpurun_out/pmc
