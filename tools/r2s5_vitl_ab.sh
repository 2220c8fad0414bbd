set -o pipefail
OUT=gpurun_out/r2s5_vitl_ab; mkdir -p $OUT
for rep in 1 2; do
  for g in def 4; do
    if [ $g = def ]; then unset VPF_GEMM_GROUP VPF_GEMM_KERNEL; else export VPF_GEMM_GROUP=4 VPF_GEMM_KERNEL=1; fi
    timeout -k 10 600 python bench.py --arch vit_large_patch14_336 --steps 2 --warmup 1 --cpu-seconds 0 --kernel-frames 1 > $OUT/l_${g}_r$rep.log 2>&1 || exit $?
    echo "vitl defaults=$g rep=$rep $(tail -1 $OUT/l_${g}_r$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels"]; print(d["ms_per_step"], " ".join("%s %.3f" % (n, k[n]["avg_ms"]) for n in ("gemm_qkv","gemm_proj","gemm_fc1","gemm_fc2")))')"
  done
done
