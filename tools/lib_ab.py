"""Same-process A/B of one C-ABI entry point between two builds of the library (design aid, GPU box only): the product
libvpf.so (bound by vitparticlefiltertracker_amd._lib) and another build loaded side by side with RTLD_LOCAL (default:
the lab build, tools/gemm_lab -> libvpf_lab.so, whose MX8 GEMM / attention are the round-3 snapshots). Both get the
same device buffers; interleaved rounds, HIP-event medians, outputs compared bit for bit.

Cases: bf16_qkv / bf16_proj / bf16_fc1 / bf16_fc2 (vpf_gemm_bf16 with the encoder's epilogues), mx8_fc1 (LN + GELU, MX8-only output: FC2's A operand), mx8_fc2 / mx8_proj (residual + planes + the MX8 copy of h),
mx8_qkv (LN fold, bf16 out), quant (vpf_quantize_mx8 of a bf16 [M][768] tensor), attn (bf16 attention, N = 197),
attn577 (bf16 attention at ViT-L/14 @ 336's N = 577, 16 heads).

usage: python tools/lib_ab.py [rounds] [cases] [other_lib]      env AB_M (rows, default 4096*197)
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vitparticlefiltertracker_amd import _lib as E  # noqa: E402
from vitparticlefiltertracker_amd import ops  # noqa: E402,F401

V = torch.ops.vpf


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    cases = sys.argv[2].split(",") if len(sys.argv) > 2 else ["mx8_fc1", "mx8_fc2", "mx8_qkv", "quant", "attn"]
    other = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "vitparticlefiltertracker_amd", "libvpf_lab.so")
    P = E.lib()
    O = ctypes.CDLL(other, mode=ctypes.RTLD_LOCAL)
    for L in (P, O):
        L.vpf_gemm_mx8.argtypes = E.SIGNATURES["vpf_gemm_mx8"]
        L.vpf_quantize_mx8.argtypes = E.SIGNATURES["vpf_quantize_mx8"]
        L.vpf_attention_bf16.argtypes = E.SIGNATURES["vpf_attention_bf16"]
        L.vpf_gemm_bf16.argtypes = E.SIGNATURES["vpf_gemm_bf16"]
    M = int(os.environ.get("AB_M", 4096 * 197))
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    st = torch.cuda.current_stream().cuda_stream
    pt = E.ptr
    for case in cases:
        outs = {}
        if case in ("attn", "attn577"):
            # attn: ViT-B/16 @ 224 (N = 197, 12 heads, the key-pipelined kernel); attn577: ViT-L/14 @ 336 (N = 577,
            # 16 heads, the key-streamed kernel), 4096 particles unless AB_M says otherwise
            N, H = (197, 12) if case == "attn" else (577, 16)
            B = M // 197
            qkv = (torch.randn(B, N, 3 * 64 * H, device=dev, generator=g) * 1.5).to(torch.bfloat16)
            bufs = {k: torch.empty(B, N, 64 * H, device=dev, dtype=torch.bfloat16) for k in ("product", "other")}

            def call(L, k):
                return L.vpf_attention_bf16(pt(qkv), pt(bufs[k]), B, N, H, 64, 0.125, N, st)
            flop = 4.0 * B * H * N * N * 64
        elif case == "quant":
            x = (torch.randn(M, 768, device=dev, generator=g) * 3).to(torch.bfloat16)
            bufs = {k: ops.mx8_empty(M, 768, dev) for k in ("product", "other")}

            def call(L, k):
                q, s = bufs[k]
                return L.vpf_quantize_mx8(pt(x), 768, M, 768, 1, pt(q), q.stride(0), pt(s), s.shape[1], st)
            flop = 0.0
        elif case.startswith("bf16_"):
            # the bf16 GEMMs with their product epilogues: qkv (LN fold), proj / fc2 (residual in place + statistics
            # planes), fc1 (LN fold + GELU); LN statistics planes of the A operand itself
            N, K, epi = {"bf16_qkv": (2304, 768, E.VPF_EPI_LN), "bf16_proj": (768, 768, E.VPF_EPI_BIAS_RESIDUAL),
                         "bf16_fc1": (3072, 768, E.VPF_EPI_LN_GELU),
                         "bf16_fc2": (768, 3072, E.VPF_EPI_BIAS_RESIDUAL)}[case]
            a = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
            w = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16)
            bias = torch.rand(N, device=dev, generator=g) * 0.1
            colsum = w.float().sum(1).contiguous()
            af = a.float().view(M, K // 64, 64)
            planes = torch.stack([af.sum(2), (af * af).sum(2)], 2).transpose(0, 1).contiguous()   # [K/64][M][2]
            res0 = (torch.rand(M, N, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
            resid = epi == E.VPF_EPI_BIAS_RESIDUAL
            bufs = {}
            for k in ("product", "other"):
                out = res0.clone() if resid else torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                bufs[k] = (out, torch.empty(N // 64, M, 2, device=dev) if resid else None)

            def call(L, k, reset=False):
                out, so = bufs[k]
                if resid and reset:
                    out.copy_(res0)
                return L.vpf_gemm_bf16(pt(a), K, pt(w), pt(bias), pt(out) if resid else None, None, 0,
                                       None if resid else pt(planes), None if resid else pt(colsum), pt(out), N, M, N, K,
                                       epi, 0 if resid else K // 64, 1e-6, pt(so) if resid else None, None, 0, None, 0,
                                       st)
            flop = 2.0 * M * N * K
        else:
            N, K = {"mx8_fc1": (3072, 768), "mx8_fc2": (768, 3072), "mx8_qkv": (2304, 768), "mx8_proj": (768, 768)}[case]
            a = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
            w = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16)
            a8, as8 = ops.mx8_empty(M, K, dev)
            w8, ws8 = ops.mx8_empty(N, K, dev)
            V.quantize_mx8_(a, 1, a8, as8)
            V.quantize_mx8_(w, 1, w8, ws8)
            bias = torch.rand(N, device=dev, generator=g) * 0.1
            colsum = w.float().sum(1).contiguous()
            Pn = 0                                     # the product's LN form: one combined {mean, rstd} plane
            planes = torch.rand(M, 2, device=dev, generator=g) + 0.5
            res0 = (torch.rand(M, N, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
            bufs = {}
            for k in ("product", "other"):
                out = res0.clone() if case in ("mx8_fc2", "mx8_proj") else torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                q8, s8 = ops.mx8_empty(M, N, dev)
                bufs[k] = (out, q8, s8, torch.empty((N + 63) // 64, M, 2, device=dev))
            epi = {"mx8_fc1": E.VPF_EPI_LN_GELU, "mx8_fc2": E.VPF_EPI_BIAS_RESIDUAL, "mx8_qkv": E.VPF_EPI_LN,
                   "mx8_proj": E.VPF_EPI_BIAS_RESIDUAL}[case]

            def call(L, k, reset=False):
                out, q8, s8, pl = bufs[k]
                fc1, fc2 = case == "mx8_fc1", case in ("mx8_fc2", "mx8_proj")
                if fc2 and reset:                      # the residual is read in place: same input for the bit check
                    out.copy_(res0)
                return L.vpf_gemm_mx8(pt(a8), a8.stride(0), pt(as8), as8.shape[1], pt(w8), pt(ws8), pt(bias),
                                      pt(out) if fc2 else None, None if fc2 else pt(planes),
                                      None if fc2 else pt(colsum), None if fc1 else pt(out), N, pt(q8) if fc1 or fc2 else None,
                                      q8.stride(0), pt(s8) if fc1 or fc2 else None, s8.shape[1], M, N, K, epi,
                                      0 if fc2 else Pn, 1e-6, pt(pl) if fc2 else None, st)
            flop = 2.0 * M * N * K
        for k, L in (("product", P), ("other", O)):
            assert (call(L, k, reset=True) if case.startswith(("mx8", "bf16")) else call(L, k)) == 0, (case, k)
        torch.cuda.synchronize()
        def snap(k):   # the outputs the call writes
            b = bufs[k]
            if case == "mx8_fc1":
                b = b[1:3]
            elif case == "mx8_qkv" or case in ("bf16_qkv", "bf16_fc1"):
                b = b[:1]
            return [t.clone() for t in (b if isinstance(b, (tuple, list)) else (b,)) if t is not None]
        same = all(torch.equal(x, y) for x, y in zip(snap("product"), snap("other")))
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        times = {"product": [], "other": []}
        for r in range(rounds):
            for k, L in ((("product", P), ("other", O)) if r % 2 == 0 else (("other", O), ("product", P))):
                ev[0].record()
                for _ in range(3):
                    call(L, k)
                ev[1].record()
                torch.cuda.synchronize()
                times[k].append(ev[0].elapsed_time(ev[1]) / 3)
        for k in times:
            t = sorted(times[k])
            med = t[len(t) // 2]
            extra = f"  {flop / med / 1e9:.1f} TFLOP/s" if flop else ""
            print(f"{case:8s} {k:8s} M={M}  median {med:.4f} ms (min {t[0]:.4f}){extra}", flush=True)
        print(f"{case:8s} outputs bit-identical: {same}", flush=True)
        del bufs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
