set -o pipefail
OUT=gpurun_out/r2s5_v4; mkdir -p $OUT
bash tools/gpu_session.sh r2s5_v4 bench prof || exit $?
for p in 2048 1024 512; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --particles $p > $OUT/bench_p$p.log 2>&1 || exit $?
  tail -1 $OUT/bench_p$p.log | cut -c1-200
done
timeout -k 10 600 python bench.py --dtype fp8 --frame 1080x1920 --particles 8192 --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/bench_c5share.log 2>&1 || exit $?
tail -1 $OUT/bench_c5share.log | cut -c1-200
timeout -k 10 900 python bench.py --arch vit_large_patch14_336 --steps 2 --warmup 1 --cpu-seconds 0 > $OUT/bench_vitl.log 2>&1 || exit $?
tail -1 $OUT/bench_vitl.log | cut -c1-200
