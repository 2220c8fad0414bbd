mkdir -p gpurun_out/r2s5_rccl
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/rccl_probe.py > gpurun_out/r2s5_rccl/probe.log 2>&1
echo "rc=$?"
grep -v "amdgpu.ids" gpurun_out/r2s5_rccl/probe.log | tail -25
