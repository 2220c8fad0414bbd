set -o pipefail
OUT=gpurun_out/r2s5_ab_cpb; mkdir -p $OUT
for rep in 1 2; do
  for v in def cpb3 cpb5 cpb6 cpb7; do
    if [ $v = def ]; then unset VPF_LIB_PATH; else export VPF_LIB_PATH=$PWD/ab_libs/libvpf_$v.so; fi
    timeout -k 10 300 python bench.py --steps 8 --warmup 2 --cpu-seconds 0 --kernel-frames 2 > $OUT/b_${v}_r$rep.log 2>&1 || exit $?
    echo "variant=$v rep=$rep $(tail -1 $OUT/b_${v}_r$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels"]; print(d["ms_per_step"], "attn", k["attention"]["avg_ms"])')"
  done
done
