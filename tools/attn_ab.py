"""Same-process A/B of the bf16 attention launch variants at the configs[1] shape (4096 particles x 12 heads, N = 197):
rounds of (variant A, variant B, ...) launches, HIP-event time per launch, medians per variant.

Lab library only (VPF_LIB_PATH=vitparticlefiltertracker_amd/libvpf_lab.so: the product library has no variants).
Variants: "tune=<k>" = its vpf_attention_tune(k) (0 = the persistent chunk ring, 1 = the one-unit key-pipelined kernel,
2 / 3 = other ring geometries, 4 / 5 = the ring's load-only / compute-only probes); anything else is a set of
environment settings the lab library reads (VPF_ATTN_TAIL16, VPF_ATTN_TAIL, VPF_ATTN_MODE, VPF_ATTN_LAB).

    python tools/attn_ab.py [--particles 4096] [--rounds 15] [--n 197] [tune=1 tune=0 ...]
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--particles", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--n", type=int, default=197)
    ap.add_argument("--heads", type=int, default=12)
    ap.add_argument("variants", nargs="*", default=["tune=1", "tune=0", "tune=2", "tune=3"])
    args = ap.parse_args()
    import torch

    from vitparticlefiltertracker_amd import _lib, ops  # noqa: F401
    L = _lib.lib()
    P, N, H = args.particles, args.n, args.heads
    D = 64 * H
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = (torch.randn(P, N, 3 * D, device="cuda", generator=g) * 1.5).to(torch.bfloat16)
    outs = {v: torch.empty(P, N, D, device="cuda", dtype=torch.bfloat16) for v in args.variants}
    times = {v: [] for v in args.variants}

    def launch(v):
        for kv in v.split(","):
            k, val = kv.split("=")
            if k == "tune":
                assert L.vpf_attention_tune(int(val)) == 0
            else:
                os.environ[k] = val
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        torch.ops.vpf.attention(qkv, H, N, outs[v])
        e.record()
        return s, e

    for v in args.variants:          # warm-up
        launch(v)
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        evs = [(v, *launch(v)) for v in args.variants]
        torch.cuda.synchronize()
        for v, s, e in evs:
            times[v].append(s.elapsed_time(e))
    flop = 4.0 * P * H * N * N * 64
    for v in args.variants:
        med = statistics.median(times[v])
        print(f"{v:32s} median {med:.4f} ms  min {min(times[v]):.4f}  {flop / med / 1e9:.1f} TFLOP/s", flush=True)
    base = outs[args.variants[0]]
    for v in args.variants[1:]:
        d = (outs[v].float() - base.float()).abs()
        print(f"{v}: max |diff| vs {args.variants[0]} = {d.max().item():.3e}, rows differing: "
              f"{int((d.amax(dim=2) > 0).sum().item())} of {P * N}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
