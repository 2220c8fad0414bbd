set -o pipefail
OUT=gpurun_out/r2s5_ab_kern; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 -k "gemm or tracker or multirank or smoke or cls" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for kk in def 1; do
    for p in 4096 512; do
      if [ $kk = def ]; then unset VPF_GEMM_KERNEL; else export VPF_GEMM_KERNEL=$kk; fi
      timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --kernel-frames 1 --particles $p > $OUT/b_k${kk}_p${p}_r$rep.log 2>&1 || exit $?
      echo "kernel=$kk p=$p rep=$rep $(tail -1 $OUT/b_k${kk}_p${p}_r$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels"]; print(d["ms_per_step"], "qkv", k["gemm_qkv"]["avg_ms"])')"
    done
  done
done
