set -o pipefail
OUT=gpurun_out/r2s5_gloo; mkdir -p $OUT
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --cpu-seconds 0 --dist-backend gloo > $OUT/bench_gloo2.log 2>&1 || exit $?
tail -1 $OUT/bench_gloo2.log | cut -c1-400
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 3 --warmup 1 --cpu-seconds 0 --dist-backend gloo --particles 4096 > $OUT/bench_gloo4.log 2>&1 || exit $?
tail -1 $OUT/bench_gloo4.log | cut -c1-400
