"""Diagnostic (GPU box): persistent GEMM kernel 14 vs kernel 1 mismatch map per 256x256 tile, LN epilogue."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitparticlefiltertracker_amd import _lib
from vitparticlefiltertracker_amd import ops as vpf
L = _lib.lib()
dev = "cuda:0"
for (M, N, K, epi, parts) in [(256 * 300, 2304, 768, 5, 12), (256 * 300, 2304, 768, 4, 0), (256 * 300, 2304, 768, 0, 0), (256 * 300, 2304, 768, 4, 12)]:
    torch.manual_seed(0)
    a = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device=dev) * 0.1
    colsum = w.float().sum(1).contiguous()
    if parts:
        stats = torch.stack([torch.randn(parts, M, device=dev) * 3.0, torch.rand(parts, M, device=dev) * 60 + 40], 2).contiguous()
    else:
        stats = torch.stack([torch.rand(M, device=dev) * 0.2 - 0.1, torch.rand(M, device=dev) + 0.5], 1).contiguous()
    outs = {}
    for k in (1, 13, 14):
        assert L.vpf_gemm_tune(k, -1) == 0
        out = torch.full((M, N), 7.0, device=dev, dtype=torch.bfloat16)
        if epi == 4:
            vpf.gemm(a, w, bias, None, None, 0, stats, colsum, epi, out, parts, 1e-6)
        else:
            vpf.gemm(a, w, bias, None, None, 0, None, None, epi, out)
        torch.cuda.synchronize()
        outs[k] = out
    L.vpf_gemm_tune(1, -1)
    bad = (outs[1].view(torch.int16) != outs[14].view(torch.int16))
    print('k13 bad', int((outs[1].view(torch.int16) != outs[13].view(torch.int16)).sum()))
    tm, tn = M // 256, N // 256
    t = bad.view(tm, 256, tn, 256).sum((1, 3))
    print(f"M={M} N={N} epi={epi} parts={parts}: bad elements {int(bad.sum())}, bad tiles {int((t > 0).sum())} of {tm * tn}")
    bt = (t > 0).nonzero().tolist()
    print("  first bad tiles (tm, tn):", bt[:20])
    if bt:
        r = bad.view(tm, 256, tn, 256)[bt[0][0], :, bt[0][1], :]
        print("  rows bad in first bad tile:", r.any(1).nonzero().flatten().tolist()[:40])
        print("  cols bad in first bad tile:", r.any(0).nonzero().flatten().tolist()[:40])
        i, j = bt[0]
        print("  sample ref/got:", outs[1][i * 256, j * 256:j * 256 + 4].tolist(), outs[14][i * 256, j * 256:j * 256 + 4].tolist())
