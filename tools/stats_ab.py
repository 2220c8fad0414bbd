"""A/B (design aid, GPU box): residual-stream statistics via the row_stats pass ({mean, rstd} rows, P = 0)
against statistics planes written by the producing GEMM (stats_out) and combined by the LN-folded consumer
(P = 3), on the ViT-B/16 shapes at 4096 particles, interleaved rounds in one process."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitparticlefiltertracker_amd import _lib, ops  # noqa: E402,F401

vpf = torch.ops.vpf
M, D, F = 4096 * 197, 768, 3072
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
h = (torch.randn(M, D, device=dev, generator=g)).to(torch.bfloat16)
x = (torch.randn(M, D, device=dev, generator=g)).to(torch.bfloat16)
Wp = (torch.randn(D, D, device=dev, generator=g) / D ** 0.5).to(torch.bfloat16)
W1 = (torch.randn(F, D, device=dev, generator=g) / D ** 0.5).to(torch.bfloat16)
bp = torch.zeros(D, device=dev)
b1 = torch.zeros(F, device=dev)
c1 = W1.float().sum(1)
hid = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
st = torch.empty(M, 2, device=dev)
planes = torch.empty(12, M, 2, device=dev)
RES, LNG = _lib.VPF_EPI_BIAS_RESIDUAL, _lib.VPF_EPI_LN_GELU


def old():
    vpf.gemm(x, Wp, bp, h, None, 0, None, None, RES, h)
    vpf.row_stats(h, 1e-6, st)
    vpf.gemm(h, W1, b1, None, None, 0, st, c1, LNG, hid)


def new():
    vpf.gemm_stats_(x, Wp, bp, h, None, 0, RES, h, planes)
    vpf.gemm(h, W1, b1, None, None, 0, planes, c1, LNG, hid, 12, 1e-6)


parts = {
    "proj": lambda: vpf.gemm(x, Wp, bp, h, None, 0, None, None, RES, h),
    "proj+stats_out": lambda: vpf.gemm_stats_(x, Wp, bp, h, None, 0, RES, h, planes),
    "row_stats": lambda: vpf.row_stats(h, 1e-6, st),
    "fc1 P=0": lambda: vpf.gemm(h, W1, b1, None, None, 0, st, c1, LNG, hid),
    "fc1 P=12": lambda: vpf.gemm(h, W1, b1, None, None, 0, planes, c1, LNG, hid, 12, 1e-6),
    "old chain": old,
    "new chain": new,
}
for f in parts.values():
    f()
torch.cuda.synchronize()
res = {k: [] for k in parts}
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for _ in range(7):
    for k, f in parts.items():
        ev[0].record()
        for _ in range(3):
            f()
        ev[1].record()
        torch.cuda.synchronize()
        res[k].append(ev[0].elapsed_time(ev[1]) / 3)
for k, v in res.items():
    v.sort()
    print(f"{k:16s} median {v[len(v) // 2]:.3f} ms  (min {v[0]:.3f})", flush=True)
