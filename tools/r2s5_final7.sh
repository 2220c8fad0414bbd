set -o pipefail
bash tools/gpu_session.sh r2s5_final7 tests smoke bench prof || exit $?
OUT=gpurun_out/r2s5_final7
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --particles 512 > $OUT/bench_p512.log 2>&1 || exit $?
tail -1 $OUT/bench_p512.log | cut -c1-200
