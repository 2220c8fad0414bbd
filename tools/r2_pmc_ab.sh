#!/bin/bash
# One PMC pass per counter group over tools/gemm_ab.py (kernels given in KERNS), kernel-trace on.
OUT=gpurun_out/${1:-r2pmc}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export PYTHONUNBUFFERED=1
run() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o p --output-format csv -- python3 tools/gemm_ab.py 1 ${SHAPES:-fc1,fc2} ${KERNS:-1,5} > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run sq2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_COUNT
run tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
echo pmc-done
