set -o pipefail
PYTEST_K="splitk or cls or tracker or multirank or gemm" bash tools/gpu_session.sh r2s5_v5 tests || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --particles 512 > gpurun_out/r2s5_v5/bench_p512.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/r2s5_v5/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r2s5_v5/bench_p512.log | cut -c1-200; tail -1 gpurun_out/r2s5_v5/bench.log | cut -c1-200
