#!/bin/bash
# kernel 7 (four-wave, AGPR accumulators): GEMM tests with every epilogue, then the A/B against kernel 1
OUT=gpurun_out/${1:-r2w4}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
VPF_GEMM_KERNEL=7 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_mx8.py -k "gemm and not mx8_plain and not mx8_layernorm and not mx8_q8_output and not mx8_residual" > $OUT/pytest_k7.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_k7.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/gemm_ab.py ${ROUNDS:-7} ${SHAPES:-qkv,proj,fc1,fc2} ${KERNS:-1,7} > $OUT/ab.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $OUT/ab.log; exit $rc
