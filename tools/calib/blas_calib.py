"""Design aid: hipBLASLt (torch.matmul / F.linear) and libvpf GEMM TFLOP/s on the ViT-B/16 encoder shapes
at 4096 particles, same process, interleaved rounds. Not part of the product."""
import sys, time
import torch
sys.path.insert(0, ".")
from vitparticlefiltertracker_amd import ops

M = 4096 * 197
shapes = {"qkv": (2304, 768), "proj": (768, 768), "fc1": (3072, 768), "fc2": (768, 3072)}
dev = "cuda"
torch.manual_seed(0)
res = {}
for name, (N, K) in shapes.items():
    a = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    b = torch.zeros(N, device=dev, dtype=torch.float32)
    bb = b.to(torch.bfloat16)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * M * N * K
    cands = {
        "hipblaslt_linear": lambda: torch.nn.functional.linear(a, w, bb),
        "hipblaslt_mm": lambda: torch.mm(a, w.t(), out=out),
        "vpf": lambda: ops.gemm(a, w, b, None, None, 0, None, None, 0, out),
    }
    for f in cands.values():
        f()
    torch.cuda.synchronize()
    for _ in range(5):
        for cname, f in cands.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                f()
            e1.record()
            torch.cuda.synchronize()
            res.setdefault((name, cname), []).append(e0.elapsed_time(e1) / 5)
    for cname in cands:
        t = sorted(res[(name, cname)])[2]
        print(f"{name:5s} {cname:18s} {t:7.3f} ms  {fl / t / 1e9:7.1f} TFLOP/s", flush=True)
    del a, w, out
