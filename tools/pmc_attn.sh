#!/bin/bash
# PMC passes over the attention kernel alone (tools/attn_probe.py, product library): where its waves spend their time.
# One rocprofv3 --pmc pass per counter group (tools/pmc_pick.py packs them within the per-block limits), each under its
# own kill-timeout. usage: tools/pmc_attn.sh <outdir> [P] [N] [H]
OUT=$1; P=${2:-4096}; N=${3:-577}; H=${4:-16}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1
echo "list rc=$?"
for grp in $(python3 tools/pmc_pick.py $OUT/counters.txt); do
  name=${grp%%:*}; ctr=${grp#*:}
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -d $OUT/$name -o p --output-format csv -- python3 tools/attn_probe.py $P 3 $N $H > $OUT/$name.log 2>&1
  rc=$?; echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
echo pmc-done
