"""ORACLE (test infrastructure only): ctypes binding of oracle/pf_oracle.c. See oracle/__init__.py.

Each function cites the SPEC.md section it restates; the reference has no implementation to cite
beyond README.md:8 ("Particle Filter ... probabilistic algorithms for accurate state estimation").
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle_pf.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
                os.path.join(_HERE, "pf_oracle.c")):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        i64, u64, u32, f32, i32 = ctypes.c_int64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_float, ctypes.c_int
        L.orc_philox4x32_10.argtypes = [P, P, P]
        L.orc_logf.argtypes = [f32]; L.orc_logf.restype = f32
        L.orc_expf.argtypes = [f32]; L.orc_expf.restype = f32
        L.orc_sincos2pi.argtypes = [f32, P, P]
        L.orc_predict.argtypes = [P, P, P, i64, i64, u64, u32, f32, f32, f32, f32, f32, f32, f32]
        L.orc_crop_patches.argtypes = [P, i32, i32, P, P, P, i64, f32, f32, i32, i32, i32, P, P, P]
        L.orc_shard_stats.argtypes = [P, P, P, P, i64, P, P]
        L.orc_position.argtypes = [u64, u64, u64, u32]; L.orc_position.restype = u64
        L.orc_resample_U.argtypes = [u64, u32]; L.orc_resample_U.restype = u32
        L.orc_resample.argtypes = [P, i64, u32, P, P]
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> ctypes.c_void_p:
    assert a.flags["C_CONTIGUOUS"]
    return ctypes.c_void_p(a.ctypes.data)


def philox4x32_10(ctr, key) -> np.ndarray:
    """SPEC S1."""
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    k = np.ascontiguousarray(key, dtype=np.uint32)
    out = np.zeros(4, np.uint32)
    lib().orc_philox4x32_10(_ptr(c), _ptr(k), _ptr(out))
    return out


def norm_affine(mean, std) -> Tuple[np.ndarray, np.ndarray]:
    """SPEC S3: a_c = f32(f32(1/255) * f32(1/std_c)), b_c = f32(-mean_c * f32(1/std_c))."""
    inv255 = np.float32(1.0) / np.float32(255.0)
    a = np.zeros(3, np.float32)
    b = np.zeros(3, np.float32)
    for c in range(3):
        inv_std = np.float32(1.0) / np.float32(std[c])
        a[c] = np.float32(inv255 * inv_std)
        b[c] = np.float32(-np.float32(mean[c]) * inv_std)
    return a, b


def predict(particles: np.ndarray, global_begin: int, seed: int, frame: int, motion_std, width: int,
            height: int, scale_range) -> None:
    """SPEC S2, in place on a float32[3][n] SoA array."""
    assert particles.dtype == np.float32 and particles.shape[0] == 3 and particles.flags["C_CONTIGUOUS"]
    n = particles.shape[1]
    xs, ys, ss = (particles[i] for i in range(3))
    lib().orc_predict(_ptr(xs), _ptr(ys), _ptr(ss), n, int(global_begin), int(seed) & (2**64 - 1),
                      int(frame), float(motion_std[0]), float(motion_std[1]), float(motion_std[2]),
                      float(width), float(height), float(scale_range[0]), float(scale_range[1]))


def crop_patches(frame: np.ndarray, particles: np.ndarray, box_wh, img_size: int, patch: int, kp: int,
                 mean, std) -> np.ndarray:
    """SPEC S3: float32[n * g*g][kp] im2col patch matrix."""
    frame = np.ascontiguousarray(frame, dtype=np.uint8)
    H, W, C = frame.shape
    assert C == 3
    particles = np.ascontiguousarray(particles, dtype=np.float32)
    n = particles.shape[1]
    g = img_size // patch
    out = np.empty((n * g * g, kp), np.float32)
    a, b = norm_affine(mean, std)
    xs, ys, ss = (np.ascontiguousarray(particles[i]) for i in range(3))
    lib().orc_crop_patches(_ptr(frame), H, W, _ptr(xs), _ptr(ys), _ptr(ss), n, float(box_wh[0]),
                           float(box_wh[1]), img_size, patch, kp, _ptr(a), _ptr(b), _ptr(out))
    return out


def shard_stats(Q: np.ndarray, particles: np.ndarray) -> Tuple[int, np.ndarray]:
    """SPEC S6 partial sums of one shard: (T_r, [sum Qx, sum Qy, sum Qs]) — index-order fp64."""
    Q = np.ascontiguousarray(Q, dtype=np.int64)
    particles = np.ascontiguousarray(particles, dtype=np.float32)
    T = ctypes.c_int64(0)
    sums = np.zeros(3, np.float64)
    xs, ys, ss = (np.ascontiguousarray(particles[i]) for i in range(3))
    lib().orc_shard_stats(_ptr(Q), _ptr(xs), _ptr(ys), _ptr(ss), Q.shape[0], ctypes.byref(T), _ptr(sums))
    return int(T.value), sums


def estimate(Q: np.ndarray, particles: np.ndarray) -> Tuple[float, float, float]:
    """SPEC S6: (x, y, s) = sum Q_i state_i / T, uniform when T == 0."""
    T, sums = shard_stats(Q, particles)
    if T == 0:
        return tuple(float(v) for v in particles.astype(np.float64).mean(axis=1))
    return float(sums[0] / T), float(sums[1] / T), float(sums[2] / T)


def resample_U(seed: int, frame: int) -> int:
    """SPEC S1: U = r0 of Philox(ctr=(0, frame, 1, 0))."""
    return int(lib().orc_resample_U(int(seed) & (2**64 - 1), int(frame)))


def position(j: int, T: int, P: int, U: int) -> int:
    """SPEC S7 pos_j (64-bit exact)."""
    return int(lib().orc_position(j, T, P, U))


def resample(Q: np.ndarray, U: int) -> np.ndarray:
    """SPEC S7: int32[P] ancestors of the global systematic resample."""
    Q = np.ascontiguousarray(Q, dtype=np.int64)
    P = Q.shape[0]
    anc = np.empty(P, np.int32)
    scratch = np.empty(P, np.int64)
    lib().orc_resample(_ptr(Q), P, int(U), _ptr(anc), _ptr(scratch))
    return anc


def weights_to_Q(sim: np.ndarray, lam: float, bits: int) -> np.ndarray:
    """SPEC S5 from fp32 cosine similarities: Q = floor(exp(lam*(min(sim, 1)-1)) * 2^bits); a non-finite
    similarity gets Q = 0 (vpf layernorm.hip k_cls_weight)."""
    sim = np.asarray(sim, np.float32)
    w = np.array([lib().orc_expf(float(np.float32(np.float32(lam) * (min(s, np.float32(1.0)) - np.float32(1.0)))))
                  if np.isfinite(s) else 0.0 for s in sim], dtype=np.float32)
    return np.floor(w.astype(np.float64) * float(2 ** bits)).astype(np.int64)
