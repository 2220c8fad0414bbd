set -o pipefail
bash tools/gpu_session.sh r2s5_final5 tests smoke || exit $?
OUT=gpurun_out/r2s5_final5
for rep in 1 2 3; do
  for v in new old; do
    if [ $v = new ]; then unset VPF_GEMM_KERNEL VPF_GEMM_GROUP VPF_CLS_SPLITK; else export VPF_GEMM_KERNEL=1 VPF_GEMM_GROUP=4 VPF_CLS_SPLITK=0; fi
    for p in 4096 512; do
      timeout -k 10 300 python bench.py --steps 8 --warmup 2 --cpu-seconds 0 --kernel-frames 1 --particles $p > $OUT/b_${v}_p${p}_r$rep.log 2>&1 || exit $?
      echo "defaults=$v p=$p rep=$rep $(tail -1 $OUT/b_${v}_p${p}_r$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
    done
  done
done
unset VPF_GEMM_KERNEL VPF_GEMM_GROUP VPF_CLS_SPLITK
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > $OUT/bench_default.log 2>&1 || exit $?
tail -1 $OUT/bench_default.log | cut -c1-200
