"""A/B (GPU box): the particle-crop gather at P particles of a 224x224 frame (64x64 template, scales 0.5-2):
LDS-staged source window (default) vs global taps (VPF_CROP_LDS=0). usage: python tools/crop_ab.py [P] [rounds]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitparticlefiltertracker_amd import ops  # noqa: E402,F401
from vitparticlefiltertracker_amd.ops import rgba_workspace  # noqa: E402
from vitparticlefiltertracker_amd.vit import norm_affine  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 9
H = W = 224
rng = np.random.default_rng(0)
fd = torch.from_numpy(rng.integers(0, 256, (H, W, 3), dtype=np.uint8)).cuda()
pt = np.empty((3, P), np.float32)
pt[0], pt[1], pt[2] = rng.uniform(60, 160, P), rng.uniform(60, 160, P), rng.uniform(0.8, 1.25, P)
pd = torch.from_numpy(pt).cuda()
ws = rgba_workspace((H, W), "cuda")
ab = norm_affine((0.5,) * 3, (0.5,) * 3)
out = torch.empty(P * 196, 768, device="cuda", dtype=torch.bfloat16)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
times = {"0": [], "1": []}
res = {}
for r in range(rounds):
    for v in (("0", "1") if r % 2 == 0 else ("1", "0")):
        os.environ["VPF_CROP_LDS"] = v
        torch.ops.vpf.crop_patches(fd, ws, pd, [64.0, 64.0], 224, 16, ab, out)
        ev[0].record()
        for _ in range(5):
            torch.ops.vpf.crop_patches(fd, ws, pd, [64.0, 64.0], 224, 16, ab, out)
        ev[1].record()
        torch.cuda.synchronize()
        times[v].append(ev[0].elapsed_time(ev[1]) / 5)
        res[v] = out.clone() if r == 0 else res.get(v)
print("outputs equal:", torch.equal(res["0"], res["1"]))
for v in ("0", "1"):
    t = sorted(times[v])
    print(f"VPF_CROP_LDS={v} P={P}: median {t[len(t) // 2]:.4f} ms (min {t[0]:.4f})", flush=True)
