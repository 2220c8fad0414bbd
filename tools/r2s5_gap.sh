set -o pipefail
OUT=gpurun_out/r2s5_gap; mkdir -p $OUT
timeout -k 10 300 python tools/gap_probe.py 512 30 > $OUT/gap512.log 2>&1 || exit $?
timeout -k 10 300 python tools/gap_probe.py 4096 10 > $OUT/gap4096.log 2>&1 || exit $?
grep "P=" $OUT/gap512.log $OUT/gap4096.log
