#!/bin/bash
# Tile-order group sweep (kernel 1, A-panel group g) on the four encoder shapes, one process per shape.
OUT=gpurun_out/${1:-r2grp}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
for s in qkv fc1 proj fc2; do
  timeout -k 10 300 python -u tools/gemm_ab.py ${ROUNDS:-5} $s ${VARS:-1:1,1:2,1:3,1:4,1:6,1:8,1:12,1:16} > $OUT/$s.log 2>&1
  rc=$?; echo "$s rc=$rc"; grep -v amdgpu.ids $OUT/$s.log | grep median; [ $rc -eq 0 ] || exit $rc
done
