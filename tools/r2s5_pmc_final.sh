set -o pipefail
OUT=gpurun_out/r2s5_pmc_final; mkdir -p $OUT
bash tools/gpu_session.sh r2s5_pmc_final pmc || exit $?
for rep in 1 2; do
  for g in def 16; do
    if [ $g = def ]; then unset VPF_GEMM_GROUP; else export VPF_GEMM_GROUP=$g; fi
    timeout -k 10 300 python bench.py --steps 6 --warmup 2 --cpu-seconds 0 --kernel-frames 2 > $OUT/b_${g}_r$rep.log 2>&1 || exit $?
    echo "fc1group=$g rep=$rep $(tail -1 $OUT/b_${g}_r$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels"]; print(d["ms_per_step"], "fc1", k["gemm_fc1"]["avg_ms"], "traffic", d["roofline"]["traffic"])')"
  done
done
