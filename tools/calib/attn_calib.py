"""Design aid (round 1): attention kernels (VPF_ATTN_MODE 0 = whole-image per-(particle, head) workgroups, 2 = key-pipelined
double-buffered) on the ViT-B/16 shape at 4096 particles, interleaved rounds in one process. The modes are read only by
the lab build (tools/gemm_lab -> libvpf_lab.so, loaded with VPF_LIB_PATH); the product library has no mode switch."""
import os, sys
import torch
sys.path.insert(0, ".")
from vitparticlefiltertracker_amd import ops

B, N, H = int(os.environ.get("ATT_B", 4096)), 197, int(os.environ.get("ATT_H", 12))
MODES = sys.argv[1].split(",") if len(sys.argv) > 1 else ["0", "1"]
D = 64 * H
torch.manual_seed(0)
qkv = (torch.randn(B, N, 3 * D, device="cuda") * 1.5).to(torch.bfloat16)
out = torch.empty(B, N, D, device="cuda", dtype=torch.bfloat16)
bytes_ = qkv.numel() * 2 + out.numel() * 2
fl = 4.0 * B * H * N * N * 64
res = {}
for _ in range(2):
    for m in MODES:
        os.environ["VPF_ATTN_MODE"] = m
        ops.attention(qkv, H, N, out)
torch.cuda.synchronize()
for _ in range(7):
    for m in MODES:
        os.environ["VPF_ATTN_MODE"] = m
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            ops.attention(qkv, H, N, out)
        e1.record()
        torch.cuda.synchronize()
        res.setdefault(m, []).append(e0.elapsed_time(e1) / 5)
for m, v in res.items():
    t = sorted(v)[len(v) // 2]
    print(f"mode {m}: {t:.3f} ms  {bytes_ / t / 1e6:.0f} GB/s  {fl / t / 1e9:.0f} TFLOP/s (min {min(v):.3f})", flush=True)
