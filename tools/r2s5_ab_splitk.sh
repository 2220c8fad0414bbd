set -o pipefail
OUT=gpurun_out/r2s5_ab_splitk; mkdir -p $OUT
for rep in 1 2; do
  for sk in 1 0; do
    for p in 512 4096; do
      VPF_CLS_SPLITK=$sk timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --kernel-frames 1 --particles $p > $OUT/b_sk${sk}_p${p}_r$rep.log 2>&1 || exit $?
      echo "sk=$sk p=$p rep=$rep $(tail -1 $OUT/b_sk${sk}_p${p}_r$rep.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
    done
  done
done
