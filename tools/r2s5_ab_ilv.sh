set -o pipefail
OUT=gpurun_out/r2s5_ab_ilv; mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 -k "crop or tracker or smoke" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in def ilv8 ilv10 ilv12; do
    if [ $v = def ]; then unset VPF_LIB_PATH; else export VPF_LIB_PATH=$PWD/ab_libs/libvpf_$v.so; fi
    timeout -k 10 600 python tools/gemm_ab.py 5 fc1,proj,fc2 1 > $OUT/ab_${v}_r$rep.log 2>&1 || exit $?
    grep median $OUT/ab_${v}_r$rep.log | sed "s/^/$v r$rep /"
  done
done
