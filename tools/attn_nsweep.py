"""Design aid (GPU box): the N <= 256 attention kernel's time per launch at several token counts, 4096 particles x 12
heads, to separate work-proportional cost from the strip-per-SIMD imbalance (round 6). At N = 197 a unit has 6 full
32-query strips + the 16-query tail strip on 8 waves (2 per SIMD): the busiest SIMD carries 2 full strips against an
average of 1.625; N = 224 (7 full strips) has the same busiest-SIMD load with 1.08x the work, N = 256 (8 strips)
2 strips per SIMD evenly with 1.41x the work, N = 192 (6 strips) the same busiest load with 0.94x the work. If the
busiest SIMD binds, t(224) ~ t(197) and t(256) / t(197) ~ 8/7 (its 8 key steps against 7); if the work binds, the
ratios follow the work.
usage: python tools/attn_nsweep.py [reps] [N,N,...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitparticlefiltertracker_amd import ops  # noqa: E402,F401

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
Ns = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [160, 192, 197, 208, 224, 240, 256]
P, H = 4096, 12
D = 64 * H
g = torch.Generator(device="cuda").manual_seed(0)
for N in Ns:
    qkv = (torch.randn(P, N, 3 * D, device="cuda", generator=g) * 1.5).to(torch.bfloat16)
    out = torch.empty(P, N, D, device="cuda", dtype=torch.bfloat16)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
    torch.ops.vpf.attention(qkv, H, N, out)
    for r in range(reps):
        ev[2 * r].record()
        torch.ops.vpf.attention(qkv, H, N, out)
        ev[2 * r + 1].record()
    torch.cuda.synchronize()
    ts = sorted(ev[2 * r].elapsed_time(ev[2 * r + 1]) for r in range(reps))
    t = ts[len(ts) // 2]
    full, tail = N // 32, N % 32
    strips = full + (0.5 if 0 < tail <= 16 else (1 if tail else 0))     # 16-query tail strip ~ half a strip
    steps = (N + 31) // 32
    work = strips * steps                                                 # strip-steps per unit
    bytes_ = P * N * 3 * D * 2 + P * N * D * 2
    print(f"N={N:4d}  {t:.4f} ms  strip-steps/unit {work:6.1f}  ms per 1k strip-steps/unit {1e3 * t / work:.3f}  "
          f"HBM {bytes_ / t / 1e6:.0f} GB/s", flush=True)
    del qkv, out
