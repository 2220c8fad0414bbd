"""Same-process A/B (round 5): an LN-folded GEMM reading the producer's statistics planes itself (P planes DMA'd into
its LDS and combined per row in the epilogue) against vpf_stats_combine (a separate {mean, rstd} pass) + the GEMM with
stats_parts = 0. ViT-B/16 shapes at 4096 particles (QKV N = 2304, FC1 N = 3072; K = D = 768, P = 12), or ViT-L/14 @ 336
with --vitl (K = 1024, P = 16: the GEMM itself then runs kernel 1's wide form); --mx8: the fp8 path's MX8 QKV (LN fold,
bf16 out) instead. Outputs compared bit for bit.

    python tools/planes_ab.py [rounds] [--vitl | --mx8]
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitparticlefiltertracker_amd import ops  # noqa: E402,F401

V = torch.ops.vpf


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 7
    vitl = "--vitl" in sys.argv
    D, N_tok = (1024, 577) if vitl else (768, 197)
    M = 4096 * N_tok
    P = D // 64
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    h = (torch.randn(M, D, device=dev, generator=g) + 0.3).to(torch.bfloat16)
    planes = torch.empty(P, M, 2, device=dev)
    hv = h.view(M, P, 64).float()
    planes[:, :, 0] = hv.sum(2).t()
    planes[:, :, 1] = (hv * hv).sum(2).t()
    st = torch.empty(M, 2, device=dev)
    if "--mx8" in sys.argv:
        N = 3 * D
        W = (torch.randn(N, D, device=dev, generator=g) / D ** 0.5).to(torch.bfloat16)
        bias = 0.1 * torch.randn(N, device=dev, generator=g)
        h8 = ops.mx8_empty(M, D, dev)
        V.quantize_mx8_(h, 1, *h8)
        w8 = ops.mx8_empty(N, D, dev)
        V.quantize_mx8_(W, 1, *w8)
        colsum = ops.mx8_dequantize(*w8).sum(dim=1).contiguous()
        outs = {k: torch.empty(M, N, device=dev, dtype=torch.bfloat16) for k in ("planes", "combine")}

        def run8(k):
            if k == "planes":
                V.gemm_mx8(*h8, *w8, bias, None, planes, colsum, 4, outs[k], P, 1e-6)
            else:
                V.stats_combine_(planes, D, 1e-6, st)
                V.gemm_mx8(*h8, *w8, bias, None, st, colsum, 4, outs[k], 0, 1e-6)
        times = {k: [] for k in outs}
        for k in outs:
            run8(k)
        torch.cuda.synchronize()
        for r in range(rounds):
            for k in (list(outs) if r % 2 == 0 else list(outs)[::-1]):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run8(k)
                e1.record()
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1))
        for k in outs:
            print(f"mx8 qkv {k:8s} median {statistics.median(times[k]):.4f} ms (min {min(times[k]):.4f})", flush=True)
        print(f"mx8 qkv: outputs bit-identical: {torch.equal(outs['planes'], outs['combine'])}", flush=True)
        return 0
    for name, N, epi in (("qkv", 3 * D, 4), ("fc1", 4 * D, 5)):
        W = (torch.randn(N, D, device=dev, generator=g) / D ** 0.5).to(torch.bfloat16)
        bias = 0.1 * torch.randn(N, device=dev, generator=g)
        colsum = W.float().sum(1).contiguous()
        outs = {k: torch.empty(M, N, device=dev, dtype=torch.bfloat16) for k in ("planes", "combine")}

        def run(k):
            if k == "planes":
                V.gemm(h, W, bias, None, None, 0, planes, colsum, epi, outs[k], P, 1e-6)
            else:
                V.stats_combine_(planes, D, 1e-6, st)
                V.gemm(h, W, bias, None, None, 0, st, colsum, epi, outs[k])
        times = {k: [] for k in outs}
        for k in outs:
            run(k)
        torch.cuda.synchronize()
        for r in range(rounds):
            for k in (list(outs) if r % 2 == 0 else list(outs)[::-1]):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run(k)
                e1.record()
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1))
        for k in outs:
            print(f"{name} {'vitl' if vitl else 'vitb'} {k:8s} median {statistics.median(times[k]):.4f} ms "
                  f"(min {min(times[k]):.4f})", flush=True)
        print(f"{name}: outputs bit-identical: {torch.equal(outs['planes'], outs['combine'])}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
