"""GPU (MI355X): the HIP ViT forward pinned DIRECTLY to the transformers-generated golden vectors.

tests/golden/vit_*.npz hold transformers' ViTModel CLS features (final LayerNorm) for seeded weights and pixels
(tests/golden/make_golden.py; SURVEY.md §8c pin (2)). The CPU suite pins the oracle to them
(test_oracle_vit.py); here the product path itself, ViTEngine on libvpf.so, runs the same pixels: the seeded weights
are rebuilt (perturb_affine=True, as the generator used them), the normalised pixel tensor is cut into the im2col
patch rows the crop kernel would write (K order c*p^2 + ky*p + kx, zero-padded to the GEMM's K), and the patch GEMM,
the encoder and the final LayerNorm run on the GPU. No oracle code sits between the HIP output and the golden.

Bars: fp32 parity mode rtol 1e-4 (atol 1e-4 for near-zero components); the bf16 product mode cosine >= 0.999 per
image (the bf16 contract of SURVEY.md §8c)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
DEV = "cuda"
CASES = ["vit_tiny_patch16_224", "vit_base_patch16_224", "vit_large_patch14_336"]


def _pixels(seed: int, batch: int, size: int) -> torch.Tensor:
    """The generator's pixel tensor (make_golden.pixels_for): uniform in [-1, 1), [B, 3, S, S]."""
    g = torch.Generator().manual_seed(seed)
    return torch.rand(batch, 3, size, size, generator=g) * 2.0 - 1.0


def _hip_cls_features(name: str, dtype: str):
    from vitparticlefiltertracker_amd.config import ARCHS
    from vitparticlefiltertracker_amd.vit import ViTEngine
    from vitparticlefiltertracker_amd.weights import make_vit_weights
    d = np.load(os.path.join(GOLD, f"vit_{name}.npz"), allow_pickle=False)
    arch = ARCHS[name]
    B = int(d["batch"])
    w = make_vit_weights(arch, seed=int(d["weight_seed"]), perturb_affine=True)
    eng = ViTEngine(arch, w, dtype, DEV, B)
    px = _pixels(int(d["pixel_seed"]), B, arch.img_size)
    p, g = arch.patch, arch.grid
    rows = px.reshape(B, 3, g, p, g, p).permute(0, 2, 4, 1, 3, 5).reshape(B * g * g, 3 * p * p)
    patches = torch.zeros(B * g * g, arch.patch_kp)
    patches[:, : 3 * p * p] = rows
    eng.patches[: B * arch.n_patches].copy_(patches.to(DEV, eng.dt))
    eng._embed_rest(B)
    eng.encoder(B)
    from vitparticlefiltertracker_amd import ops  # noqa: F401
    dummy_t = torch.zeros(arch.dim, device=DEV, dtype=torch.float32)
    torch.ops.vpf.cls_weight(eng.h[:B], eng.ng, eng.nb, arch.ln_eps, dummy_t, 0.0, 0, eng.Q[:B], eng.feat[:B], None)
    torch.cuda.synchronize()
    return eng.feat[:B].cpu().numpy().astype(np.float64), d["cls"].astype(np.float64)


@pytest.mark.parametrize("name", CASES)
def test_hip_fp32_forward_matches_transformers_golden(name):
    got, ref = _hip_cls_features(name, "fp32")
    assert got.shape == ref.shape and np.all(np.isfinite(got))
    err = np.abs(got - ref)
    print(f"{name} fp32: max |HIP - transformers| = {err.max():.3e}, max rel {np.max(err / (np.abs(ref) + 1e-6)):.3e}")
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("name", CASES)
def test_hip_bf16_forward_matches_transformers_golden(name):
    got, ref = _hip_cls_features(name, "bf16")
    assert got.shape == ref.shape and np.all(np.isfinite(got))
    cos = (got * ref).sum(1) / (np.linalg.norm(got, axis=1) * np.linalg.norm(ref, axis=1))
    print(f"{name} bf16: cosine to transformers per image {np.round(cos, 6).tolist()}")
    assert cos.min() >= 0.999, cos
