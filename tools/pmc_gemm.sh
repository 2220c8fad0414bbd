#!/bin/bash
# PMC passes over the bf16 GEMMs alone (tools/gemm_ab.py, product library): which unit bounds the K loop.
# One rocprofv3 --pmc pass per counter group (MI355X_MICROARCH.md §rocprofv3 PMC slots: <= 8 SQ, 4 TCC, 4 TCP, 2 TA,
# 2 TD, 2 GRBM per pass), each under its own kill-timeout; the counter list of this box first.
# usage: tools/pmc_gemm.sh <outdir> [shapes] [variants]
OUT=$1; SHAPES=${2:-fc1,fc2}; VARS=${3:-1}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1
echo "list rc=$?"
run() {  # name, counters (comma separated)
  local name=$1 ctr=$2
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -d $OUT/$name -o p --output-format csv -- python3 tools/gemm_ab.py 1 $SHAPES $VARS > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
for grp in $(python3 tools/pmc_pick.py $OUT/counters.txt); do
  name=${grp%%:*}; ctr=${grp#*:}
  run $name $ctr
done
echo pmc-done
