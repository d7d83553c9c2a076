set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_bench.py --rows 10000000 --variant device_hist_blocks=256 --variant device_hist_blocks=128 --variant device_hist_blocks=192 --variant device_hist_blocks=160 > gpurun_out/ab10m.log 2>&1 || exit $?
tail -2 gpurun_out/ab10m.log
timeout -k 10 200 python -u scripts/ab_bench.py --rows 1250000 --variant device_hist_blocks=0 --variant device_hist_blocks=64 --variant device_hist_blocks=96 --variant device_hist_blocks=128 > gpurun_out/ab1m.log 2>&1 || exit $?
tail -2 gpurun_out/ab1m.log
