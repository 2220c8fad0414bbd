"""A/B timing of the libvpf GEMM kernels on the ViT-B/16 encoder shapes with their real epilogues
(design aid, GPU box only): kernel 1 (k_gemm_bf16, one 256x256 tile per 512-thread workgroup) against
kernel 2 (k_gemm_bf16_t2, two 256x128-tile workgroups per CU), interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24), random operands, outputs compared bit for bit.

usage: python tools/gemm_ab.py [rounds] [shapes comma list] [variants comma list: k or k:group]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitparticlefiltertracker_amd import _lib  # noqa: E402
from vitparticlefiltertracker_amd import ops as vpf  # noqa: E402

E = _lib
GROUP = int(os.environ.get("AB_GROUP", -1))
SHAPES = {  # name: (N, K, epilogue)
    "qkv": (2304, 768, E.VPF_EPI_LN),
    "proj": (768, 768, E.VPF_EPI_BIAS_RESIDUAL),
    "fc1": (3072, 768, E.VPF_EPI_LN_GELU),
    "fc2": (768, 3072, E.VPF_EPI_BIAS_RESIDUAL),
    "proj_bias": (768, 768, E.VPF_EPI_BIAS),
    "fc1_bias": (3072, 768, E.VPF_EPI_BIAS),
    "fc2_bias": (768, 3072, E.VPF_EPI_BIAS),
    "patch": (768, 768, E.VPF_EPI_PATCH),   # ViT-B/16 patch embed (196 patch rows per crop, CLS-offset output rows)
    # ViT-L/14 @ 336 (configs[3]; run with AB_M=2363392 = 4096 x 577)
    "qkv_l": (3072, 1024, E.VPF_EPI_LN),
    "proj_l": (1024, 1024, E.VPF_EPI_BIAS_RESIDUAL),
    "fc1_l": (4096, 1024, E.VPF_EPI_LN_GELU),
    "fc2_l": (1024, 4096, E.VPF_EPI_BIAS_RESIDUAL),
}


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    names = sys.argv[2].split(",") if len(sys.argv) > 2 and sys.argv[2] else list(SHAPES)
    # variants "k" or "k:g" (kernel k with tile-order group g)
    kerns = sys.argv[3].split(",") if len(sys.argv) > 3 else ["1", "2"]

    def tune(v):
        k, _, g = v.partition(":")
        return L.vpf_gemm_tune(int(k), int(g) if g else GROUP)
    M = int(os.environ.get("AB_M", 4096 * 197))
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(0)
    L = _lib.lib()
    for name in names:
        N, K, epi = SHAPES[name]
        a = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16)
        bias = torch.rand(N, device=dev, generator=g) * 0.1
        colsum = w.float().sum(1).contiguous()
        stats = torch.stack([torch.rand(M, device=dev, generator=g) * 0.2 - 0.1,
                             torch.rand(M, device=dev, generator=g) + 0.5], 1).contiguous()
        patch = epi == E.VPF_EPI_PATCH
        g2 = 196
        Mp = M // g2 * g2 if patch else M
        if patch:
            a = a[:Mp]
        pos = torch.rand(g2 + 1, N, device=dev, generator=g) * 0.1 if patch else None
        res0 = (torch.rand(Mp // g2 * (g2 + 1) if patch else M, N, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        outs = {}
        flop = 2.0 * M * N * K
        ln = epi in (E.VPF_EPI_LN, E.VPF_EPI_LN_GELU)
        resid = epi == E.VPF_EPI_BIAS_RESIDUAL

        def run(out):
            if patch:
                vpf.gemm(a, w, bias, None, pos, g2, None, None, epi, out)
                return
            vpf.gemm(a, w, bias, out if resid else None, None, 0, stats if ln else None, colsum if ln else None,
                     epi, out)

        for k in kerns:
            assert tune(k) == 0
            out = res0.clone()
            run(out)
            torch.cuda.synchronize()
            outs[k] = out
        ref = outs[kerns[0]]
        for k in kerns[1:]:
            bad = (outs[k].view(torch.int16) != ref.view(torch.int16)).sum().item()
            print(f"{name} kernel {k} mismatches vs kernel {kerns[0]}: {bad}", flush=True)
        times = {k: [] for k in kerns}
        out = res0.clone()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for r in range(rounds):
            for k in (kerns if r % 2 == 0 else kerns[::-1]):   # alternate the order: no position bias
                tune(k)
                ev[0].record()
                for _ in range(3):
                    run(out)
                ev[1].record()
                torch.cuda.synchronize()
                times[k].append(ev[0].elapsed_time(ev[1]) / 3)
        for k in kerns:
            t = sorted(times[k])
            med = t[len(t) // 2]
            print(f"{name:5s} kernel {k}  M={M} N={N} K={K}  median {med:.3f} ms  {flop / med / 1e9:.1f} TFLOP/s  "
                  f"(min {t[0]:.3f})", flush=True)
        del a, w, res0, outs, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
