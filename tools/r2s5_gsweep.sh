set -o pipefail
OUT=gpurun_out/r2s5_gsweep; mkdir -p $OUT
timeout -k 10 900 python tools/gemm_ab.py 9 fc1 1:4,1:8,1:16,1:24,1:32,1:48 > $OUT/fc1.log 2>&1 || exit $?
timeout -k 10 900 python tools/gemm_ab.py 9 proj,fc2 1:1,1:2,1:3 > $OUT/projfc2.log 2>&1 || exit $?
grep median $OUT/fc1.log $OUT/projfc2.log
