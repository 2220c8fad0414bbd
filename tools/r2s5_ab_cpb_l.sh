set -o pipefail
OUT=gpurun_out/r2s5_ab_cpb_l; mkdir -p $OUT
for rep in 1 2; do
  for v in def cpb4; do
    if [ $v = def ]; then unset VPF_LIB_PATH; else export VPF_LIB_PATH=$PWD/ab_libs/libvpf_$v.so; fi
    timeout -k 10 600 python bench.py --arch vit_large_patch14_336 --steps 2 --warmup 1 --cpu-seconds 0 --kernel-frames 1 > $OUT/l_${v}_r$rep.log 2>&1 || exit $?
    echo "vitl variant=$v rep=$rep $(tail -1 $OUT/l_${v}_r$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels"]; print(d["ms_per_step"], "attn", k["attention"]["avg_ms"])')"
    timeout -k 10 300 python bench.py --dtype fp8 --steps 5 --warmup 2 --cpu-seconds 0 --kernel-frames 1 > $OUT/f_${v}_r$rep.log 2>&1 || exit $?
    echo "fp8 variant=$v rep=$rep $(tail -1 $OUT/f_${v}_r$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels"]; print(d["ms_per_step"], "attn", k["attention"]["avg_ms"])')"
  done
done
