set -o pipefail
OUT=gpurun_out/r2s5_fc1pp; mkdir -p $OUT
timeout -k 10 900 python tools/gemm_ab.py 11 fc1 1:16,5:16,5:8,1:8 > $OUT/fc1.log 2>&1 || exit $?
AB_M=100864 timeout -k 10 900 python tools/gemm_ab.py 11 fc1 1:16,5:16,5:8,1:8 > $OUT/fc1_512.log 2>&1 || exit $?
grep median $OUT/fc1.log $OUT/fc1_512.log
