set -o pipefail
OUT=gpurun_out/r2s5_mx8_fc1g; mkdir -p $OUT
for rep in 1 2 3; do
  for g in 4 1 2; do
    VPF_GEMM_GROUP=$g timeout -k 10 300 python bench.py --dtype fp8 --steps 4 --warmup 2 --cpu-seconds 0 --kernel-frames 2 > $OUT/g${g}_r$rep.log 2>&1 || exit $?
    echo "fp8 group=$g rep=$rep $(tail -1 $OUT/g${g}_r$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels"]; print(d["ms_per_step"], " ".join("%s %.4f" % (n, k[n]["avg_ms"]) for n in ("gemm_qkv","gemm_proj","gemm_fc1","gemm_fc2")))')"
  done
done
