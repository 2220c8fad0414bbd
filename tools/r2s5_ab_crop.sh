set -o pipefail
OUT=gpurun_out/r2s5_ab_crop; mkdir -p $OUT
for rep in 1 2; do
  for v in def crop10240 crop6144 crop4608; do
    if [ $v = def ]; then unset VPF_LIB_PATH; else export VPF_LIB_PATH=$PWD/ab_libs/libvpf_$v.so; fi
    for p in 4096 512; do
      timeout -k 10 300 python bench.py --steps 6 --warmup 2 --cpu-seconds 0 --kernel-frames 3 --particles $p > $OUT/b_${v}_p${p}_r$rep.log 2>&1 || exit $?
      echo "crop=$v p=$p rep=$rep $(tail -1 $OUT/b_${v}_p${p}_r$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels"]; print(d["ms_per_step"], "crop", k["crop_patches"]["avg_ms"])')"
    done
  done
done
