#!/bin/bash
# PMC passes over tools/calib/blas_calib.py (hipBLASLt vs libvpf, same shapes); one counter group per pass.
OUT=gpurun_out/calib_pmc; mkdir -p $OUT
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o p --output-format csv -- python3 tools/calib/blas_calib.py > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run tcc_hit TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
echo pmc-done
