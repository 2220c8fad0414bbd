mkdir -p gpurun_out/r2s2
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_kernels.py tests/test_gpu_vit_tracker.py -k "sharded or cancellation or edge_rows or cls_weight or upload or stats_planes" > gpurun_out/r2s2/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/r2s2/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --cpu-seconds 0 --dist-backend gloo > gpurun_out/r2s2/bench_gloo2.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/r2s2/bench_gloo2.log | cut -c1-700
