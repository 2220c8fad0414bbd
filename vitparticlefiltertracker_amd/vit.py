"""ViT feature extractor on the HIP path (the reference's "Vision Transformer (ViT)
... feature extraction", /root/reference/README.md:7).

`ViTEngine` holds the device weights and every activation buffer for a fixed particle batch and runs one
frame's forward as a fixed chain of `torch.ops.vpf.*` launches on the current HIP stream:

    crop+im2col -> patch GEMM (+bias +pos, scattered into token rows) -> CLS rows
    L x [ LN1 -> QKV GEMM(+bias) -> attention -> proj GEMM(+bias +residual, in place on h)
          LN2 -> FC1 GEMM(+bias +GELU) -> FC2 GEMM(+bias +residual, in place on h) ]
    final LN of the CLS rows -> cosine to the template -> int64 fixed-point weights Q

Because every buffer is preallocated and no launch synchronises, the chain is captured once into a HIP
graph (`torch.cuda.CUDAGraph`, which is a hipGraph on ROCm) and replayed per frame (`capture=True`).

HBM layout (bf16 mode, P particles, N tokens, D width, F MLP width):
  h   [P][N][D]   residual stream (bf16)          x   [P][N][D]   LN output / attention output
  qkv [P][N][3D]  (3, heads, 64) column order      hid [P][N][F]   GELU(FC1) (also hosts the im2col patches)
Weights are [out][in] (K-contiguous rows) bf16 with fp32 biases / LayerNorm affines / cls / pos.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from . import _lib
from . import ops  # noqa: F401  (registers torch.ops.vpf)
from .config import ViTArch

vpf = torch.ops.vpf


def norm_affine(mean, std):
    """SPEC S3 per-channel affine {a0,a1,a2,b0,b1,b2} in fp32 (same rounding as the oracle)."""
    one = torch.tensor(1.0, dtype=torch.float32)
    inv255 = one / torch.tensor(255.0, dtype=torch.float32)
    a, b = [], []
    for c in range(3):
        inv_std = one / torch.tensor(float(std[c]), dtype=torch.float32)
        a.append(float((inv255 * inv_std).item()))
        b.append(float((-torch.tensor(float(mean[c]), dtype=torch.float32) * inv_std).item()))
    return a + b


class KernelTimer:
    """HIP-event timing of individual launches on the current stream (eager mode only; bench.py)."""

    def __init__(self):
        self.pending = []     # (name, start, end)

    def __call__(self, name, fn, *args):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        fn(*args)
        e.record()
        self.pending.append((name, s, e))

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for name, s, e in self.pending:
            d = out.setdefault(name, [0, 0.0])
            d[0] += 1
            d[1] += s.elapsed_time(e)
        return {k: {"launches": v[0], "total_ms": v[1], "avg_ms": v[1] / v[0]} for k, v in out.items()}


def _run(timer, name, fn, *args):
    if timer is None:
        fn(*args)
    else:
        timer(name, fn, *args)


class ViTEngine:
    def __init__(self, arch: ViTArch, weights: Dict[str, torch.Tensor], dtype: str, device, batch: int,
                 mean=(0.5, 0.5, 0.5), std=(0.5, 0.5, 0.5)):
        if not torch.cuda.is_available():
            raise _lib.VPFError("ViTEngine needs a HIP device (the product path has no CPU fallback)")
        _lib.lib()  # fail loudly now if libvpf.so is missing
        self.arch = arch
        self.device = torch.device(device)
        self.dt = torch.bfloat16 if dtype == "bf16" else torch.float32
        self.batch = int(batch)
        self.norm_ab = norm_affine(mean, std)
        A = arch
        D, F, N = A.dim, A.mlp, A.tokens
        dev, dt = self.device, self.dt

        def mat(t):
            return t.to(dev, dt).contiguous()

        def f32(t):
            return t.to(dev, torch.float32).contiguous()

        wpe = weights["patch_embed.weight"].reshape(D, A.patch_k)
        wpe_p = torch.zeros(D, A.patch_kp)
        wpe_p[:, :A.patch_k] = wpe
        self.w_pe = mat(wpe_p)
        self.b_pe = f32(weights["patch_embed.bias"])
        self.cls = f32(weights["cls_token"])
        self.pos = f32(weights["pos_embed"])
        self.layers = []
        for l in range(A.depth):
            p = f"blocks.{l}."
            self.layers.append({
                "n1g": f32(weights[p + "norm1.weight"]), "n1b": f32(weights[p + "norm1.bias"]),
                "wqkv": mat(weights[p + "attn.qkv.weight"]), "bqkv": f32(weights[p + "attn.qkv.bias"]),
                "wproj": mat(weights[p + "attn.proj.weight"]), "bproj": f32(weights[p + "attn.proj.bias"]),
                "n2g": f32(weights[p + "norm2.weight"]), "n2b": f32(weights[p + "norm2.bias"]),
                "wfc1": mat(weights[p + "mlp.fc1.weight"]), "bfc1": f32(weights[p + "mlp.fc1.bias"]),
                "wfc2": mat(weights[p + "mlp.fc2.weight"]), "bfc2": f32(weights[p + "mlp.fc2.bias"]),
            })
        self.ng = f32(weights["norm.weight"])
        self.nb = f32(weights["norm.bias"])
        self._alloc(self.batch)
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.timer: Optional[KernelTimer] = None

    # ------------------------------------------------------------------ buffers
    def _alloc(self, n: int) -> None:
        A, dev, dt = self.arch, self.device, self.dt
        D, F, N = A.dim, A.mlp, A.tokens
        self.h = torch.empty(n, N, D, device=dev, dtype=dt)
        self.x = torch.empty(n, N, D, device=dev, dtype=dt)
        self.qkv = torch.empty(n, N, 3 * D, device=dev, dtype=dt)
        hid_elems = max(n * N * F, n * A.n_patches * A.patch_kp)
        self.hid_flat = torch.empty(hid_elems, device=dev, dtype=dt)
        self.hid = self.hid_flat[: n * N * F].view(n * N, F)
        self.patches = self.hid_flat[: n * A.n_patches * A.patch_kp].view(n * A.n_patches, A.patch_kp)
        self.Q = torch.empty(n, device=dev, dtype=torch.int64)
        self.feat = torch.empty(n, D, device=dev, dtype=torch.float32)
        self.sim = torch.empty(n, device=dev, dtype=torch.float32)

    # ------------------------------------------------------------------ forward pieces
    def embed(self, frame: torch.Tensor, particles: torch.Tensor, box_wh) -> None:
        A = self.arch
        n = particles.shape[1]
        patches = self.patches[: n * A.n_patches]
        T = self.timer
        _run(T, "crop_patches", vpf.crop_patches, frame, particles, [float(box_wh[0]), float(box_wh[1])],
             A.img_size, A.patch, self.norm_ab, patches)
        h = self.h[:n]
        _run(T, "gemm_patch", vpf.gemm, patches, self.w_pe, self.b_pe, None, self.pos, A.n_patches,
             _lib.VPF_EPI_PATCH, h)
        _run(T, "cls_rows", vpf.cls_rows_, h, self.cls, self.pos)

    def encoder(self, n: int) -> None:
        A = self.arch
        D, N = A.dim, A.tokens
        h = self.h[:n]
        x = self.x[:n]
        qkv = self.qkv[:n]
        hid = self.hid[: n * N]
        h2 = h.view(n * N, D)
        x2 = x.view(n * N, D)
        T = self.timer
        for L in self.layers:
            _run(T, "layernorm", vpf.layernorm, h, L["n1g"], L["n1b"], A.ln_eps, x)
            _run(T, "gemm_qkv", vpf.gemm, x2, L["wqkv"], L["bqkv"], None, None, 0, _lib.VPF_EPI_BIAS,
                 qkv.view(n * N, 3 * D))
            _run(T, "attention", vpf.attention, qkv, A.heads, x)
            _run(T, "gemm_proj", vpf.gemm, x2, L["wproj"], L["bproj"], h2, None, 0, _lib.VPF_EPI_BIAS_RESIDUAL, h2)
            _run(T, "layernorm", vpf.layernorm, h, L["n2g"], L["n2b"], A.ln_eps, x)
            _run(T, "gemm_fc1", vpf.gemm, x2, L["wfc1"], L["bfc1"], None, None, 0, _lib.VPF_EPI_BIAS_GELU, hid)
            _run(T, "gemm_fc2", vpf.gemm, hid, L["wfc2"], L["bfc2"], h2, None, 0, _lib.VPF_EPI_BIAS_RESIDUAL, h2)

    def weights_from_tokens(self, n: int, tmpl: torch.Tensor, lam: float, bits: int, want_feat: bool = False):
        _run(self.timer, "cls_weight", vpf.cls_weight, self.h[:n], self.ng, self.nb, self.arch.ln_eps, tmpl,
             float(lam), int(bits), self.Q[:n], self.feat[:n] if want_feat else None, self.sim[:n])
        return self.Q[:n]

    def features(self, frame: torch.Tensor, particles: torch.Tensor, box_wh) -> torch.Tensor:
        """LN'd CLS features [n][D] fp32 (template init, tests)."""
        n = particles.shape[1]
        assert n <= self.batch
        self.embed(frame, particles, box_wh)
        self.encoder(n)
        dummy_t = torch.zeros(self.arch.dim, device=self.device, dtype=torch.float32)
        vpf.cls_weight(self.h[:n], self.ng, self.nb, self.arch.ln_eps, dummy_t, 0.0, 0, self.Q[:n], self.feat[:n],
                       None)
        return self.feat[:n]

    def forward_weights(self, frame, particles, box_wh, tmpl, lam, bits, want_feat: bool = False):
        n = particles.shape[1]
        assert n <= self.batch
        self.embed(frame, particles, box_wh)
        self.encoder(n)
        return self.weights_from_tokens(n, tmpl, lam, bits, want_feat)
