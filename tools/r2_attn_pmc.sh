#!/bin/bash
OUT=gpurun_out/${1:-r2apmc}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export PYTHONUNBUFFERED=1
run() {
  local name=$1; shift
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o p --output-format csv -- python3 tools/attn_probe.py 4096 3 > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run sq2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_COUNT
run fetch FETCH_SIZE
run write WRITE_SIZE
timeout -k 10 120 python3 tools/attn_probe.py 4096 5 > $OUT/plain.log 2>&1; echo "plain rc=$?"; cat $OUT/plain.log | grep attention
