"""Configuration surface: the `config.yaml` schema the reference names but does not ship.

The reference's only statement about configuration is "configure the tracking parameters in the
`config.yaml` file" (/root/reference/README.md:42); the key set below is the build's contract
 and SPEC.md gives each value its meaning.
"""
from __future__ import annotations

import copy
import dataclasses
import math
import os
from typing import Any, Dict, Optional

import yaml


@dataclasses.dataclass(frozen=True)
class ViTArch:
    """A ViT architecture: image size, patch, width, depth, heads, MLP width, LayerNorm eps."""

    name: str
    img_size: int
    patch: int
    dim: int
    depth: int
    heads: int
    mlp: int
    ln_eps: float = 1e-6

    @property
    def grid(self) -> int:
        return self.img_size // self.patch

    @property
    def n_patches(self) -> int:
        return self.grid * self.grid

    @property
    def tokens(self) -> int:
        return self.n_patches + 1

    @property
    def head_dim(self) -> int:
        return self.dim // self.heads

    @property
    def patch_k(self) -> int:
        return 3 * self.patch * self.patch

    @property
    def patch_kp(self) -> int:
        """Patch-GEMM K padded to the 64-deep K-step of the HIP GEMM (SPEC S3)."""
        return (self.patch_k + 63) // 64 * 64

    def gflop_per_crop(self) -> float:
        """Algorithmic FLOPs of one crop's forward (SURVEY.md §8d formula), in GFLOP."""
        n, N, D, L, H, hd, F = self.n_patches, self.tokens, self.dim, self.depth, self.heads, self.head_dim, self.mlp
        f = 2 * (n * self.patch_k * D + L * (N * D * 3 * D + 2 * H * N * N * hd + N * D * D + 2 * N * D * F))
        return f / 1e9

    def gflop_per_crop_executed(self, cls_fused: bool = True) -> float:
        """FLOPs of the work the product path performs per crop, in GFLOP: the full forward of blocks 0..L-2, and for
        the last block only what its CLS row needs (vit.py ViTEngine.encoder: the final LayerNorm reads nothing else).
        cls_fused (csrc/cls_attn.hip): the CLS query (2 D^2), G = W'_k^T q per head (2 D^2 useful), the folded
        attention's scores and weighted row sum over N tokens (4 N D H), W'_v per head (2 D^2 useful), proj (2 D^2),
        fc1 / fc2 (4 D F). Otherwise K and V for every row (4 N D^2), the CLS query, its attention (4 H N hd) and
        the CLS row's proj / MLP. The block-diagonal GEMMs' discarded products are not counted."""
        n, N, D, L, H, hd, F = self.n_patches, self.tokens, self.dim, self.depth, self.heads, self.head_dim, self.mlp
        full_block = N * D * 3 * D + 2 * H * N * N * hd + N * D * D + 2 * N * D * F
        if cls_fused:
            last = D * D + D * D + 2 * N * D * H + D * D + D * D + 2 * D * F
        else:
            last = 2 * N * D * D + D * D + 2 * H * N * hd + D * D + 2 * D * F
        f = 2 * (n * self.patch_k * D + (L - 1) * full_block + last)
        return f / 1e9

    def gflop_per_crop_mx8(self) -> float:
        """FLOPs per crop that the fp8 path (model.dtype: fp8) runs on block-scaled MX8 MFMA, in GFLOP: QKV, FC1 and FC2
        of blocks 0..L-2, and their proj when N <= 256 (the attention then writes MX8; vit.py ViTEngine.encoder). The
        patch embedding, the attention and the last block stay bf16."""
        N, D, L, F = self.tokens, self.dim, self.depth, self.mlp
        per_block = N * D * 3 * D + 2 * N * D * F + (N * D * D if N <= 256 else 0)
        return 2 * (L - 1) * per_block / 1e9


ARCHS: Dict[str, ViTArch] = {
    "vit_tiny_patch16_224": ViTArch("vit_tiny_patch16_224", 224, 16, 192, 12, 3, 768),
    "vit_small_patch16_224": ViTArch("vit_small_patch16_224", 224, 16, 384, 12, 6, 1536),
    "vit_base_patch16_224": ViTArch("vit_base_patch16_224", 224, 16, 768, 12, 12, 3072),
    "vit_large_patch14_336": ViTArch("vit_large_patch14_336", 336, 14, 1024, 24, 16, 4096),
}


DEFAULTS: Dict[str, Any] = {
    "model": {
        "arch": "vit_base_patch16_224",
        "dtype": "bf16",                 # bf16 (product) | fp8 (MX-fp8 encoder GEMMs, configs[4]) | fp32 (parity)
        "weights": {"seed": 0},
        "mean": [0.5, 0.5, 0.5],
        "std": [0.5, 0.5, 0.5],
    },
    "particles": {
        "num": 4096,
        "motion_std": [4.0, 4.0, 0.02],
        "scale_range": [0.5, 2.0],
        "seed": 1234,
    },
    "likelihood": {"lambda": 20.0, "weight_bits": 40,
                   "template_update": 0.0},     # alpha: t <- normalise((1 - alpha) t + alpha f(estimate)); 0 = fixed
    "resample": {"method": "systematic"},
    "input": {"source": "synthetic", "frames": 32, "height": 224, "width": 224,
              "bbox0": [80, 80, 64, 64], "seed": 7,
              "bboxes": None},                # several targets (SPEC S9): [[x, y, w, h], ...]; main.py -> MultiTracker
    "distributed": {"world_size": 1},
}


def _merge(base: Dict[str, Any], over: Dict[str, Any]) -> Dict[str, Any]:
    out = copy.deepcopy(base)
    for k, v in (over or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = _merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def load_config(cfg: Optional[Any] = None) -> Dict[str, Any]:
    """Accept a path to a YAML file, a dict (partial is fine) or None; return the full config dict."""
    if cfg is None:
        user = {}
    elif isinstance(cfg, (str, os.PathLike)):
        with open(cfg, "r") as fh:
            user = yaml.safe_load(fh) or {}
    elif isinstance(cfg, dict):
        user = cfg
    else:
        raise TypeError(f"config must be a path, dict or None, got {type(cfg).__name__}")
    out = _merge(DEFAULTS, user)
    arch = out["model"]["arch"]
    if arch not in ARCHS:
        raise ValueError(f"unknown model.arch {arch!r}; known: {sorted(ARCHS)}")
    if out["model"]["dtype"] not in ("bf16", "fp8", "fp32"):
        raise ValueError("model.dtype must be 'bf16', 'fp8' or 'fp32'")
    lam = float(out["likelihood"]["lambda"])
    if not (math.isfinite(lam) and lam >= 0.0):
        raise ValueError("likelihood.lambda must be finite and >= 0 (SPEC S5)")
    if not 0.0 <= float(out["likelihood"]["template_update"]) <= 1.0:
        raise ValueError("likelihood.template_update must be in [0, 1]")
    if out["resample"]["method"] != "systematic":
        raise ValueError("only resample.method == 'systematic' is defined (SPEC S7)")
    boxes = out["input"].get("bboxes")
    if boxes is not None:
        if not isinstance(boxes, (list, tuple)) or not boxes:
            raise ValueError("input.bboxes must be a non-empty list of [x, y, w, h] boxes (or null)")
        for b in boxes:
            if not isinstance(b, (list, tuple)) or len(b) != 4 or not all(math.isfinite(float(v)) for v in b) \
                    or float(b[2]) <= 0 or float(b[3]) <= 0:
                raise ValueError(f"input.bboxes: {b!r} is not an [x, y, w, h] box with w, h > 0")
    return out


def arch_of(cfg: Dict[str, Any]) -> ViTArch:
    return ARCHS[cfg["model"]["arch"]]
