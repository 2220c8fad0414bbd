#!/bin/bash
# epilogue A/B: GEMM + MX8 + tracker tests on the default kernel, then kernel 1 (parity-row epilogue) vs 6 (original)
OUT=gpurun_out/${1:-r2epi}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_mx8.py -k "gemm" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/gemm_ab.py ${ROUNDS:-9} ${SHAPES:-qkv,proj,fc1,fc2} ${KERNS:-1,6} > $OUT/ab.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $OUT/ab.log; exit $rc
