set -o pipefail
mkdir -p gpurun_out/grp
for g in 0 4 8 16; do
  VPF_GEMM_GROUP=$g timeout -k 10 300 python tools/calib/blas_calib.py > gpurun_out/grp/g$g.log 2>&1 || exit $?
  echo "group $g"; grep vpf gpurun_out/grp/g$g.log
done
