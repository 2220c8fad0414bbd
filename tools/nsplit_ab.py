"""A/B (GPU box): a GEMM run as S launches over column slices of W (N / S columns each, into the same C with
ldc = N) against one launch: a W panel that fits the XCD's 4 MiB L2 next to the A panels in flight.
usage: python tools/nsplit_ab.py [rounds] [shape: fc1|qkv|fc2|proj] [splits comma list]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitparticlefiltertracker_amd import _lib  # noqa: E402
from vitparticlefiltertracker_amd import ops as vpf  # noqa: E402

E = _lib
SHAPES = {"fc1": (3072, 768, E.VPF_EPI_LN_GELU), "qkv": (2304, 768, E.VPF_EPI_LN), "fc2": (768, 3072, E.VPF_EPI_BIAS),
          "proj": (768, 768, E.VPF_EPI_BIAS), "fc1_bias": (3072, 768, E.VPF_EPI_BIAS)}
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
name = sys.argv[2] if len(sys.argv) > 2 else "fc1"
splits = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "1,2,3,4").split(",")]
M = int(os.environ.get("AB_M", 4096 * 197))
N, K, epi = SHAPES[name]
dev = "cuda:0"
g = torch.Generator(device=dev).manual_seed(0)
a = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
w = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16)
bias = torch.rand(N, device=dev, generator=g) * 0.1
colsum = w.float().sum(1).contiguous()
stats = torch.stack([torch.rand(M, device=dev, generator=g) * 0.2 - 0.1, torch.rand(M, device=dev, generator=g) + 0.5],
                    1).contiguous()
ln = epi in (E.VPF_EPI_LN, E.VPF_EPI_LN_GELU)
out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)


def run(S):
    n = N // S
    for s in range(S):
        c = slice(s * n, (s + 1) * n)
        vpf.gemm(a, w[c], bias[c], None, None, 0, stats if ln else None, colsum[c] if ln else None, epi, out[:, c])


ref = None
for S in splits:
    run(S)
    torch.cuda.synchronize()
    if ref is None:
        ref = out.clone()
    else:
        print(f"splits {S}: equal to splits {splits[0]}: {torch.equal(out, ref)}", flush=True)
times = {S: [] for S in splits}
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for r in range(rounds):
    for S in (splits if r % 2 == 0 else splits[::-1]):
        ev[0].record()
        for _ in range(3):
            run(S)
        ev[1].record()
        torch.cuda.synchronize()
        times[S].append(ev[0].elapsed_time(ev[1]) / 3)
flop = 2.0 * M * N * K
for S in splits:
    t = sorted(times[S])
    print(f"{name} M={M} N={N} K={K} in {S} launches: median {t[len(t) // 2]:.3f} ms  {flop / t[len(t) // 2] / 1e9:.1f} "
          f"TFLOP/s (min {t[0]:.3f})", flush=True)
