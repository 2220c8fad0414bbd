set -o pipefail
OUT=gpurun_out/r2s5_kab; mkdir -p $OUT
timeout -k 10 900 python tools/gemm_ab.py 9 qkv,fc1,proj,fc2 1,5,13 > $OUT/kab.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/kab.log
