"""bf16 vs MX-fp8 GEMM timing on the ViT-B/16 encoder shapes with the epilogues each path uses (design aid, GPU
box only). Interleaved rounds in one process; random operands.

  qkv : LN fold (12 statistics planes)                      bf16 out
  fc1 : LN fold + GELU; the fp8 path writes only the MX8 copy (FC2's A operand)
  fc2 : residual + statistics planes; the fp8 path also writes the MX8 copy of h
  proj: residual + planes (bf16 path only on both: the attention output stays bf16) — reference line

usage: python tools/mx8_ab.py [rounds] [shapes]   env AB_M (rows, default 4096*197)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitparticlefiltertracker_amd import _lib as E  # noqa: E402
from vitparticlefiltertracker_amd import ops  # noqa: E402

V = torch.ops.vpf
SHAPES = {"qkv": (2304, 768), "fc1": (3072, 768), "fc2": (768, 3072), "proj": (768, 768)}


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    names = sys.argv[2].split(",") if len(sys.argv) > 2 else list(SHAPES)
    M = int(os.environ.get("AB_M", 4096 * 197))
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    for name in names:
        N, K = SHAPES[name]
        a = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16)
        bias = torch.rand(N, device=dev, generator=g) * 0.1
        colsum = w.float().sum(1).contiguous()
        P = K // 64
        planes = torch.rand(P, M, 2, device=dev, generator=g) + 0.5
        a8, as8 = ops.mx8_empty(M, K, dev)
        w8, ws8 = ops.mx8_empty(N, K, dev)
        V.quantize_mx8_(a, 1, a8, as8)
        V.quantize_mx8_(w, 1, w8, ws8)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        pl_out = torch.empty((N + 63) // 64, M, 2, device=dev)
        q8, s8 = ops.mx8_empty(M, N, dev) if N % 128 == 0 else (None, None)
        flop = 2.0 * M * N * K

        if name == "qkv":
            f16 = lambda: V.gemm(a, w, bias, None, None, 0, planes, colsum, E.VPF_EPI_LN, out, P, 1e-6)  # noqa
            f8 = lambda: V.gemm_mx8(a8, as8, w8, ws8, bias, None, planes, colsum, E.VPF_EPI_LN, out, P, 1e-6)  # noqa
        elif name == "fc1":
            f16 = lambda: V.gemm(a, w, bias, None, None, 0, planes, colsum, E.VPF_EPI_LN_GELU, out, P, 1e-6)  # noqa
            f8 = lambda: V.gemm_mx8_q8_(a8, as8, w8, ws8, bias, planes, colsum, E.VPF_EPI_LN_GELU, q8, s8, P, 1e-6)  # noqa
        elif name == "fc2":
            f16 = lambda: V.gemm_stats_(a, w, bias, out, None, 0, E.VPF_EPI_BIAS_RESIDUAL, out, pl_out)  # noqa
            f8 = lambda: V.gemm_mx8_res_(a8, as8, w8, ws8, bias, out, pl_out, q8, s8)  # noqa
        else:
            f16 = lambda: V.gemm_stats_(a, w, bias, out, None, 0, E.VPF_EPI_BIAS_RESIDUAL, out, pl_out)  # noqa
            f8 = lambda: V.gemm_q8_(a, w, bias, out, None, 0, E.VPF_EPI_BIAS_RESIDUAL, out, pl_out, q8, s8)  # noqa
        fns = {"bf16": f16, "mx8" if name != "proj" else "bf16+q8": f8}
        for v in [x for x in os.environ.get("AB_MX8_VARIANTS", "").split(",") if x]:
            def fv(v=v, f8=f8):   # same call under VPF_MX8_VARIANT=v (read by the library at each launch)
                os.environ["VPF_MX8_VARIANT"] = v
                f8()
                os.environ.pop("VPF_MX8_VARIANT")
            fns["mx8_v" + v] = fv
        if os.environ.get("AB_NO_BF16"):   # variant A/B only: the bf16 call's own operands would cool the MALL
            fns.pop("bf16")
        for v in [x for x in os.environ.get("AB_CHECK", "").split(",") if x]:   # bit-equality of full-kernel variants
            def snap():
                torch.cuda.synchronize()
                return [t.clone() for t in (out, q8, s8) if t is not None]
            if name == "fc2":
                out.copy_(out0 := (torch.rand(M, N, device=dev, generator=g) * 2 - 1).to(torch.bfloat16))
            f8()
            ref = snap()
            if name == "fc2":
                out.copy_(out0)
            fns["mx8_v" + v]()
            got = snap()
            same = all(torch.equal(x, y) for x, y in zip(ref, got))
            print(f"{name:4s} variant {v} bit-identical to the product schedule: {same}", flush=True)
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        times = {k: [] for k in fns}
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for r in range(rounds):
            order = list(fns.items())
            for k, f in (order if r % 2 == 0 else order[::-1]):   # alternate the order: no position bias
                ev[0].record()
                for _ in range(3):
                    f()
                ev[1].record()
                torch.cuda.synchronize()
                times[k].append(ev[0].elapsed_time(ev[1]) / 3)
        for k in fns:
            t = sorted(times[k])
            med = t[len(t) // 2]
            print(f"{name:4s} {k:8s} M={M} N={N} K={K}  median {med:.3f} ms  {flop / med / 1e9:.1f} TFLOP/s "
                  f"(min {t[0]:.3f})", flush=True)
        del a, w, a8, w8, out, planes, pl_out, q8, s8
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
