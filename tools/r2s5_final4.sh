set -o pipefail
bash tools/gpu_session.sh r2s5_final4 tests smoke bench prof || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --particles 512 > gpurun_out/r2s5_final4/bench_p512.log 2>&1 || exit $?
tail -1 gpurun_out/r2s5_final4/bench_p512.log | cut -c1-200
