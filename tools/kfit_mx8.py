import os, sys, torch
sys.path.insert(0, os.getcwd())
from vitparticlefiltertracker_amd import _lib as E, ops
V = torch.ops.vpf
dev = "cuda"
M, N = 806912, 768
g = torch.Generator(device=dev).manual_seed(0)
for K in (128, 256, 768, 1536, 3072):
    a = (torch.rand(M, K, device=dev, generator=g) - 0.5).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=dev, generator=g) - 0.5) * 0.05).to(torch.bfloat16)
    bias = torch.zeros(N, device=dev)
    a8, as8 = ops.mx8_empty(M, K, dev); w8, ws8 = ops.mx8_empty(N, K, dev)
    V.quantize_mx8_(a, 1, a8, as8); V.quantize_mx8_(w, 1, w8, ws8)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    fns = {"bf16": lambda: V.gemm(a, w, bias, None, None, 0, None, None, E.VPF_EPI_BIAS, out),
           "mx8": lambda: V.gemm_mx8(a8, as8, w8, ws8, bias, None, None, None, E.VPF_EPI_BIAS, out)}
    for f in fns.values(): f()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    res = {}
    for k, f in fns.items():
        ts = []
        for _ in range(5):
            ev[0].record(); f(); f(); ev[1].record(); torch.cuda.synchronize(); ts.append(ev[0].elapsed_time(ev[1]) / 2)
        res[k] = sorted(ts)[2]
    tiles = (M // 256) * (N // 256) / 256.0
    print(f"K={K:5d}  bf16 {res['bf16']:.3f} ms ({1e3*res['bf16']/tiles:.2f} us/tile-wave)   mx8 {res['mx8']:.3f} ms ({1e3*res['mx8']/tiles:.2f} us/tile-wave)", flush=True)
    del a, w, a8, w8, out; torch.cuda.empty_cache()
