"""Generate the ViT golden vectors that pin the CPU oracle (oracle/vit.py).

The reference ships no ViT code (README.md:7) and pins no library version (requirements.txt absent,
README.md:31), so the third-party ViT implementation installed in the build container —
`transformers` 5.15.0 `ViTModel`, eager attention, random-init from a local `ViTConfig`, no network — is
the pin. This script runs ONLY in the build container (transformers does not travel to
the GPU box). It loads the build's seeded weights (vitparticlefiltertracker_amd/weights.py, with
perturbed biases / LayerNorm affines so every term is exercised) into ViTModel, runs it on seeded
pixel tensors, and stores inputs' seeds plus CLS features (final LN) and per-layer hidden-state
statistics. Weights and pixels are regenerated from their seeds by the tests; only outputs are stored.

    python tests/golden/make_golden.py [case names]
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))

from vitparticlefiltertracker_amd.config import ARCHS  # noqa: E402
from vitparticlefiltertracker_amd.weights import make_vit_weights  # noqa: E402

CASES = [
    # (arch, weight seed, pixel seed, batch)
    ("vit_tiny_patch16_224", 11, 101, 4),
    ("vit_base_patch16_224", 12, 102, 1),
    ("vit_large_patch14_336", 13, 103, 1),   # round 4 s2: configs[3]'s architecture (N = 577, D = 1024, 24 blocks)
]


def pixels_for(seed: int, batch: int, size: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return torch.rand(batch, 3, size, size, generator=g) * 2.0 - 1.0


def hf_model(arch, w):
    from transformers import ViTConfig, ViTModel
    cfg = ViTConfig(hidden_size=arch.dim, num_hidden_layers=arch.depth, num_attention_heads=arch.heads,
                    intermediate_size=arch.mlp, image_size=arch.img_size, patch_size=arch.patch,
                    layer_norm_eps=arch.ln_eps, hidden_act="gelu", qkv_bias=True,
                    hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    cfg._attn_implementation = "eager"
    m = ViTModel(cfg, add_pooling_layer=False).eval()
    D = arch.dim
    sd = {
        "embeddings.cls_token": w["cls_token"].reshape(1, 1, D),
        "embeddings.position_embeddings": w["pos_embed"].unsqueeze(0),
        "embeddings.patch_embeddings.projection.weight": w["patch_embed.weight"],
        "embeddings.patch_embeddings.projection.bias": w["patch_embed.bias"],
        "layernorm.weight": w["norm.weight"],
        "layernorm.bias": w["norm.bias"],
    }
    for l in range(arch.depth):
        b, h = f"blocks.{l}.", f"layers.{l}."
        qw, kw, vw = w[b + "attn.qkv.weight"].split(D, 0)
        qb, kb, vb = w[b + "attn.qkv.bias"].split(D, 0)
        sd.update({
            h + "attention.q_proj.weight": qw, h + "attention.q_proj.bias": qb,
            h + "attention.k_proj.weight": kw, h + "attention.k_proj.bias": kb,
            h + "attention.v_proj.weight": vw, h + "attention.v_proj.bias": vb,
            h + "attention.o_proj.weight": w[b + "attn.proj.weight"],
            h + "attention.o_proj.bias": w[b + "attn.proj.bias"],
            h + "layernorm_before.weight": w[b + "norm1.weight"], h + "layernorm_before.bias": w[b + "norm1.bias"],
            h + "layernorm_after.weight": w[b + "norm2.weight"], h + "layernorm_after.bias": w[b + "norm2.bias"],
            h + "mlp.fc1.weight": w[b + "mlp.fc1.weight"], h + "mlp.fc1.bias": w[b + "mlp.fc1.bias"],
            h + "mlp.fc2.weight": w[b + "mlp.fc2.weight"], h + "mlp.fc2.bias": w[b + "mlp.fc2.bias"],
        })
    missing, unexpected = m.load_state_dict(sd, strict=True), None
    return m


@torch.no_grad()
def main() -> None:
    import transformers
    only = set(sys.argv[1:])   # optional: the case names to (re)generate
    for name, wseed, pseed, batch in CASES:
        if only and name not in only:
            continue
        arch = ARCHS[name]
        w = make_vit_weights(arch, seed=wseed, perturb_affine=True)
        m = hf_model(arch, w)
        px = pixels_for(pseed, batch, arch.img_size)
        out = m(pixel_values=px, output_hidden_states=True)
        cls = out.last_hidden_state[:, 0].float().numpy()
        hs = out.hidden_states  # embeddings + one per layer (pre final LN)
        stats = np.array([[t.float().mean().item(), t.float().abs().mean().item(), t[:, 0].float().norm().item()]
                          for t in hs], np.float64)
        path = os.path.join(HERE, f"vit_{name}.npz")
        np.savez(path, arch=name, weight_seed=wseed, pixel_seed=pseed, batch=batch, cls=cls,
                 layer_stats=stats, transformers_version=transformers.__version__,
                 torch_version=torch.__version__)
        print(path, cls.shape, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
