"""CPU: pin the ViT oracle (oracle/vit.py) against transformers-generated golden vectors
(tests/golden/make_golden.py; SURVEY.md §8c pin (2)), and check the im2col path against the pixel path."""
import os

import numpy as np
import pytest
import torch

from oracle import pf
from oracle import vit as ovit
from vitparticlefiltertracker_amd.config import ARCHS
from vitparticlefiltertracker_amd.weights import make_vit_weights

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def pixels_for(seed: int, batch: int, size: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return torch.rand(batch, 3, size, size, generator=g) * 2.0 - 1.0


@pytest.mark.parametrize("name", ["vit_tiny_patch16_224", "vit_base_patch16_224", "vit_large_patch14_336"])
def test_vit_oracle_matches_transformers_golden(name):
    d = np.load(os.path.join(GOLD, f"vit_{name}.npz"), allow_pickle=False)
    arch = ARCHS[name]
    w = make_vit_weights(arch, seed=int(d["weight_seed"]), perturb_affine=True)
    px = pixels_for(int(d["pixel_seed"]), int(d["batch"]), arch.img_size)
    got = ovit.features_from_pixels(px, w, arch).numpy()
    ref = d["cls"]
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=2e-5)


def test_im2col_path_equals_pixel_path():
    """features_from_patches(crop_patches(identity crop)) == features_from_pixels(normalised frame)."""
    arch = ARCHS["vit_tiny_patch16_224"]
    arch = type(arch)("t2", 224, 16, 192, 2, 3, 768)
    w = make_vit_weights(arch, seed=3, perturb_affine=True)
    frame = np.random.default_rng(1).integers(0, 256, (224, 224, 3), dtype=np.uint8)
    part = np.array([[112.0], [112.0], [1.0]], np.float32)
    patches = pf.crop_patches(frame, part, (224.0, 224.0), 224, 16, arch.patch_kp, (0.5,) * 3, (0.5,) * 3)
    a, b = pf.norm_affine((0.5,) * 3, (0.5,) * 3)
    norm = (frame.astype(np.float64) * a + b).astype(np.float32).transpose(2, 0, 1)[None]
    f1 = ovit.features_from_patches(torch.from_numpy(patches), w, arch)
    f2 = ovit.features_from_pixels(torch.from_numpy(np.ascontiguousarray(norm)), w, arch)
    torch.testing.assert_close(f1, f2, rtol=1e-5, atol=1e-5)
