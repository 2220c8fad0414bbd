"""Seeded synthetic ViT weights (SPEC S4).

No pretrained checkpoint can be fetched offline (SURVEY.md §7 hard part (v)), so the tracker's
feature extractor is a random-init ViT with the timm/HF initialisation: trunc-normal(0, 0.02) for the
patch/QKV/proj/MLP matrices and the cls / position embeddings, zero biases, unit LayerNorm.
Generation order is fixed so the same seed gives the same tensors on every machine running this
torch build; the product path (vit.py) and the CPU oracle both consume this dict.

Names (timm-style): patch_embed.weight [D,3,p,p], patch_embed.bias, cls_token [D], pos_embed [N,D],
blocks.{l}.norm1.{weight,bias}, blocks.{l}.attn.qkv.{weight [3D,D], bias}, blocks.{l}.attn.proj.*,
blocks.{l}.norm2.*, blocks.{l}.mlp.fc1.{weight [F,D], bias}, blocks.{l}.mlp.fc2.*, norm.{weight,bias}.
"""
from __future__ import annotations

from typing import Dict

import torch

from .config import ViTArch


def _tn(gen: torch.Generator, *shape: int, std: float = 0.02) -> torch.Tensor:
    t = torch.empty(*shape, dtype=torch.float32)
    torch.nn.init.trunc_normal_(t, mean=0.0, std=std, a=-2 * std, b=2 * std, generator=gen)
    return t


def make_vit_weights(arch: ViTArch, seed: int = 0, perturb_affine: bool = False) -> Dict[str, torch.Tensor]:
    """Return fp32 CPU tensors. `perturb_affine=True` draws non-trivial biases and LayerNorm affines
    (tests use it to exercise every epilogue term)."""
    g = torch.Generator().manual_seed(int(seed))
    D, F, p = arch.dim, arch.mlp, arch.patch
    w: Dict[str, torch.Tensor] = {}

    def bias(n: int) -> torch.Tensor:
        return _tn(g, n, std=0.02) if perturb_affine else torch.zeros(n)

    def ln(prefix: str) -> None:
        if perturb_affine:
            w[prefix + ".weight"] = 1.0 + _tn(g, D, std=0.1)
            w[prefix + ".bias"] = _tn(g, D, std=0.05)
        else:
            w[prefix + ".weight"] = torch.ones(D)
            w[prefix + ".bias"] = torch.zeros(D)

    w["patch_embed.weight"] = _tn(g, D, 3, p, p)
    w["patch_embed.bias"] = bias(D)
    w["cls_token"] = _tn(g, D)
    w["pos_embed"] = _tn(g, arch.tokens, D)
    for l in range(arch.depth):
        b = f"blocks.{l}."
        ln(b + "norm1")
        w[b + "attn.qkv.weight"] = _tn(g, 3 * D, D)
        w[b + "attn.qkv.bias"] = bias(3 * D)
        w[b + "attn.proj.weight"] = _tn(g, D, D)
        w[b + "attn.proj.bias"] = bias(D)
        ln(b + "norm2")
        w[b + "mlp.fc1.weight"] = _tn(g, F, D)
        w[b + "mlp.fc1.bias"] = bias(F)
        w[b + "mlp.fc2.weight"] = _tn(g, D, F)
        w[b + "mlp.fc2.bias"] = bias(D)
    ln("norm")
    return w
