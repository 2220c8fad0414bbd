#!/bin/bash
# PMC passes (kernel-trace + one counter group per pass; MI355X_MICROARCH.md §rocprofv3 PMC slots)
cd "$(dirname "$0")" && make -s gemm_lab || exit 1
OUT=../../gpurun_out/pmc; mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o p --output-format csv -- ./gemm_lab 1 "$SHAPES" "$VARS" 0 > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
SHAPES=${SHAPES:-fc2,qkv}; VARS=${VARS:-V0,V3}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run sq2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA GRBM_COUNT
run tcc1 TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
run tcc2 FETCH_SIZE
run tcc3 WRITE_SIZE
echo pmc-done
