"""ORACLE (test infrastructure only): pure PyTorch-CPU fp32 functional ViT (SPEC S4). See oracle/__init__.py.

Semantics follow `transformers` ViTModel (modeling_vit.py: patch conv :42-70, eager attention with
`scaling = hd^-0.5` and fp32 softmax :164-189, pre-norm layer :257-286, final LayerNorm :385) with
layer_norm_eps = 1e-6 and exact-erf GELU (timm convention). Pinned by tests/golden/vit_*.npz which
transformers itself produced (tests/golden/make_golden.py). The reference names a "Vision
Transformer (ViT)" feature extractor (README.md:7) without an implementation.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.nn.functional as Fn


def tokens_from_patches(patches: torch.Tensor, w: Dict[str, torch.Tensor], n_part: int, n_patches: int,
                        patch_k: int) -> torch.Tensor:
    """patches: [n_part*n_patches, Kp] fp32 (im2col, SPEC S3) → tokens [n_part, N, D]."""
    D = w["cls_token"].shape[0]
    wpe = w["patch_embed.weight"].reshape(D, -1)
    emb = patches[:, :patch_k] @ wpe.t() + w["patch_embed.bias"]
    emb = emb.reshape(n_part, n_patches, D)
    cls = w["cls_token"].reshape(1, 1, D).expand(n_part, 1, D)
    h = torch.cat([cls, emb], dim=1) + w["pos_embed"].unsqueeze(0)
    return h


def block(h: torch.Tensor, w: Dict[str, torch.Tensor], l: int, heads: int, eps: float) -> torch.Tensor:
    B, N, D = h.shape
    hd = D // heads
    b = f"blocks.{l}."
    x = Fn.layer_norm(h, (D,), w[b + "norm1.weight"], w[b + "norm1.bias"], eps)
    qkv = x @ w[b + "attn.qkv.weight"].t() + w[b + "attn.qkv.bias"]
    qkv = qkv.reshape(B, N, 3, heads, hd).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    s = (q @ k.transpose(-1, -2)) * (hd ** -0.5)
    p = torch.softmax(s.float(), dim=-1)
    o = (p @ v).transpose(1, 2).reshape(B, N, D)
    h = h + (o @ w[b + "attn.proj.weight"].t() + w[b + "attn.proj.bias"])
    x = Fn.layer_norm(h, (D,), w[b + "norm2.weight"], w[b + "norm2.bias"], eps)
    m = Fn.gelu(x @ w[b + "mlp.fc1.weight"].t() + w[b + "mlp.fc1.bias"])
    h = h + (m @ w[b + "mlp.fc2.weight"].t() + w[b + "mlp.fc2.bias"])
    return h


@torch.no_grad()
def forward_tokens(h: torch.Tensor, w: Dict[str, torch.Tensor], depth: int, heads: int, eps: float,
                   capture: Optional[List[torch.Tensor]] = None) -> torch.Tensor:
    """Run the encoder on tokens [B, N, D]; return the final-LN hidden states [B, N, D]."""
    for l in range(depth):
        h = block(h, w, l, heads, eps)
        if capture is not None:
            capture.append(h.clone())
    D = h.shape[-1]
    return Fn.layer_norm(h, (D,), w["norm.weight"], w["norm.bias"], eps)


@torch.no_grad()
def features_from_pixels(pixels: torch.Tensor, w: Dict[str, torch.Tensor], arch) -> torch.Tensor:
    """pixels [B, 3, S, S] (already normalised) → CLS features [B, D] fp32 (golden-vector path)."""
    B = pixels.shape[0]
    p, g = arch.patch, arch.grid
    patches = pixels.reshape(B, 3, g, p, g, p).permute(0, 2, 4, 1, 3, 5).reshape(B * g * g, 3 * p * p)
    h = tokens_from_patches(patches, w, B, g * g, 3 * p * p)
    return forward_tokens(h, w, arch.depth, arch.heads, arch.ln_eps)[:, 0]


@torch.no_grad()
def features_from_patches(patches: torch.Tensor, w: Dict[str, torch.Tensor], arch) -> torch.Tensor:
    """im2col patches [n*g*g, Kp] fp32 (oracle.pf.crop_patches) → CLS features [n, D] fp32."""
    n = patches.shape[0] // arch.n_patches
    h = tokens_from_patches(patches, w, n, arch.n_patches, arch.patch_k)
    return forward_tokens(h, w, arch.depth, arch.heads, arch.ln_eps)[:, 0]
