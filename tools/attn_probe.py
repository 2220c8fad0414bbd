"""Design aid (GPU box): run the bf16 attention of ViT-B/16 (or any N / heads) at P particles a few times on random qkv,
for rocprofv3 PMC / kernel-trace passes over the attention kernel alone.
usage: python tools/attn_probe.py [P] [reps] [N] [H]     (ViT-L/14 @ 336: N = 577, H = 16)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitparticlefiltertracker_amd import ops  # noqa: E402,F401

P = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
N = int(sys.argv[3]) if len(sys.argv) > 3 else 197
H = int(sys.argv[4]) if len(sys.argv) > 4 else 12
D = 64 * H
g = torch.Generator(device="cuda").manual_seed(0)
qkv = (torch.randn(P, N, 3 * D, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
out = torch.empty(P, N, D, device="cuda", dtype=torch.bfloat16)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for r in range(reps):
    ev[0].record()
    torch.ops.vpf.attention(qkv, H, N, out)
    ev[1].record()
    torch.cuda.synchronize()
    print(f"attention P={P}: {ev[0].elapsed_time(ev[1]):.3f} ms", flush=True)
