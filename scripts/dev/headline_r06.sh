# headline evidence of the current tree: driver-shape bench lines, 1.25M, and a rocprofv3 kernel table
set -u
OUT=gpurun_out/headline
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 bench.py --steps 20 --warmup 2 > $OUT/b20.log 2>&1 || exit 1
echo "b20 $(tail -1 $OUT/b20.log | cut -c1-200)"
timeout -k 10 200 python3 bench.py > $OUT/b50.log 2>&1 || exit 1
echo "b50 $(tail -1 $OUT/b50.log | cut -c1-200)"
timeout -k 10 200 python3 bench.py --rows 1250000 > $OUT/b1.log 2>&1 || exit 1
echo "b1 $(tail -1 $OUT/b1.log | cut -c1-200)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run -- python3 bench.py --steps 20 --warmup 2 > $OUT/prof.log 2>&1 || exit 1
python3 scripts/prof_summary.py $OUT/prof "10M x 28, 63 leaves, final round-6 tree (bench.py --steps 20 --warmup 2)" 22 > $OUT/kernels.md
head -22 $OUT/kernels.md
