set -o pipefail
bash tools/gpu_session.sh r2s5_final6 tests smoke bench prof || exit $?
OUT=gpurun_out/r2s5_final6
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --particles 512 > $OUT/bench_p512.log 2>&1 || exit $?
tail -1 $OUT/bench_p512.log | cut -c1-200
timeout -k 10 600 python bench.py --dtype fp8 --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/bench8.log 2>&1 || exit $?
tail -1 $OUT/bench8.log | cut -c1-200
