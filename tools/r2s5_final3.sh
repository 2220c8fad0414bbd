set -o pipefail
bash tools/gpu_session.sh r2s5_final3 tests smoke bench || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --particles 512 > gpurun_out/r2s5_final3/bench_p512.log 2>&1 || exit $?
tail -1 gpurun_out/r2s5_final3/bench_p512.log | cut -c1-200
timeout -k 10 600 python bench.py --dtype fp8 --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/r2s5_final3/bench8.log 2>&1 || exit $?
tail -1 gpurun_out/r2s5_final3/bench8.log | cut -c1-200
timeout -k 10 600 python bench.py --dtype fp8 --frame 1080x1920 --particles 8192 --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/r2s5_final3/bench_c5share.log 2>&1 || exit $?
tail -1 gpurun_out/r2s5_final3/bench_c5share.log | cut -c1-200
