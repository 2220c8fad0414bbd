set -o pipefail
OUT=gpurun_out/r2s5_ab_splitk2; mkdir -p $OUT
for rep in 1 2; do
  for sk in 1 0; do
    for p in 512 4096 8192; do
      VPF_CLS_SPLITK=$sk timeout -k 10 300 python bench.py --steps 6 --warmup 2 --cpu-seconds 0 --kernel-frames 2 --particles $p > $OUT/b_sk${sk}_p${p}_r$rep.log 2>&1 || exit $?
      echo "splitk=$sk p=$p rep=$rep $(tail -1 $OUT/b_sk${sk}_p${p}_r$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels"]; print(d["ms_per_step"], "fc2_cls", k["gemm_fc2_cls"]["avg_ms"])')"
    done
  done
done
