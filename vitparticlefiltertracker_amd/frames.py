"""Synthetic frame source — the metric's input; the reference reads a "video feed or
images" (README.md:42) that it never ships. Plain-numpy readers for `.npy` clips and image directories
of raw `.npy` frames are provided for real data (no cv2 / torchvision in this image).

Clip: uint8 RGB frames; background uniform noise (numpy default_rng(seed)); a 64x64 textured target
(default_rng(seed + 1)) moving on a fixed trajectory, top-left x0 + t*v; bbox0 = (x0, y0, 64, 64).
"""
from __future__ import annotations

import glob
import os
from typing import Iterator, Tuple

import numpy as np


def target_box(t: int, bbox0=(80, 80, 64, 64), velocity=(2, 1)) -> Tuple[int, int, int, int]:
    x0, y0, w, h = bbox0
    return x0 + velocity[0] * t, y0 + velocity[1] * t, w, h


def synthetic_clip(frames: int = 32, height: int = 224, width: int = 224, bbox0=(80, 80, 64, 64), seed: int = 7,
                   velocity=(2, 1)) -> np.ndarray:
    rng = np.random.default_rng(seed)
    bg = rng.integers(0, 256, size=(height, width, 3), dtype=np.uint8)
    tex = np.random.default_rng(seed + 1).integers(0, 256, size=(bbox0[3], bbox0[2], 3), dtype=np.uint8)
    out = np.empty((frames, height, width, 3), np.uint8)
    for t in range(frames):
        f = bg.copy()
        x, y, w, h = target_box(t, bbox0, velocity)
        xa, ya = max(0, x), max(0, y)
        xb, yb = min(width, x + w), min(height, y + h)
        if xa < xb and ya < yb:
            f[ya:yb, xa:xb] = tex[ya - y: yb - y, xa - x: xb - x]
        out[t] = f
    return out


def iter_frames(source) -> Iterator[np.ndarray]:
    """Yield uint8[H][W][3] frames from a clip array, a `.npy` clip file or a directory of `.npy` frames."""
    if isinstance(source, np.ndarray):
        arr = source if source.ndim == 4 else source[None]
        for f in arr:
            yield np.ascontiguousarray(f, dtype=np.uint8)
        return
    path = os.fspath(source)
    if os.path.isdir(path):
        for p in sorted(glob.glob(os.path.join(path, "*.npy"))):
            yield np.ascontiguousarray(np.load(p, allow_pickle=False), dtype=np.uint8)
        return
    arr = np.load(path, mmap_mode="r", allow_pickle=False)
    for f in (arr if arr.ndim == 4 else arr[None]):
        yield np.ascontiguousarray(f, dtype=np.uint8)
