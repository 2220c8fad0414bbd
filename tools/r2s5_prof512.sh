set -o pipefail
OUT=gpurun_out/r2s5_prof512; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 --particles 512 > $OUT/prof.log 2>&1 || exit $?
tail -1 $OUT/prof.log | cut -c1-200
find $OUT/prof -name "*kernel_stats.csv" | head -3
