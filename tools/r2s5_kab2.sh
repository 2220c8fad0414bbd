set -o pipefail
OUT=gpurun_out/r2s5_kab2; mkdir -p $OUT
timeout -k 10 900 python tools/gemm_ab.py 15 fc1,qkv 1,5,13 > $OUT/kab.log 2>&1 || exit $?
AB_M=100864 timeout -k 10 900 python tools/gemm_ab.py 15 fc1,qkv 1,5,13 > $OUT/kab_512.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/kab.log $OUT/kab_512.log | grep median
