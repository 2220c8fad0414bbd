set -o pipefail
OUT=gpurun_out/r2s5_ab_group; mkdir -p $OUT
for rep in 1 2 3; do
  for g in def 4; do
    for p in 4096 512; do
      if [ $g = def ]; then unset VPF_GEMM_GROUP; else export VPF_GEMM_GROUP=$g; fi
      timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --kernel-frames 1 --particles $p > $OUT/b_g${g}_p${p}_r$rep.log 2>&1 || exit $?
      echo "group=$g p=$p rep=$rep $(tail -1 $OUT/b_g${g}_p${p}_r$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels"]; print(d["ms_per_step"], "proj", k["gemm_proj"]["avg_ms"], "fc2", k["gemm_fc2"]["avg_ms"])')"
    done
  done
done
