#!/bin/bash
# session-2 final: the driver's round-end tiers plus a kernel-trace profile of the headline
set -u
bash scripts/gpu_check_all.sh
