"""ORACLE (test infrastructure only; see oracle/__init__.py): numpy restatement of the MX-fp8 format used by the
fp8 path (BASELINE.json configs[4]; format in include/vpf.h "MX8 operands").

- OCP 8-bit floating point, E4M3 ("e4m3fn": bias 7, no infinities, 0x7f / 0xff = NaN, max finite 448), encoded
  here by hand with round-half-to-even (`e4m3_encode`), independent of torch's float8 cast which the CPU tests
  pin it against.
- OCP MX block scaling: one E8M0 scale (2^(byte - 127)) per 32 consecutive K values. The block exponent rule
  is the repo's (vpf.h): the smallest E with amax * 2^-E <= 448, clamped to [-127, 125], so no element
  saturates (the OCP MX spec's floor(log2 amax) - 8 would saturate the top binade).
- Scale storage: per 128-deep K-tile a plane of `lds` uint32 words, rows in bricks of 64: row r, K-block kb
  -> byte (r/16)%4 of word (r/64)*64 + kb*16 + r%16 (`scale_byte_index`).

The reference has no fp8 path (README-only, /root/reference/README.md:1-63): parity for this row is pinned by
these rules, by the OCP format's own value table, and by torch's float8_e4m3fn conversion.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

E4M3_MAX = 448.0


def e4m3_value_table() -> np.ndarray:
    """float64[256]: the value of every e4m3fn byte (NaN for 0x7f / 0xff)."""
    v = np.empty(256)
    for b in range(256):
        s = -1.0 if b & 0x80 else 1.0
        e, m = (b >> 3) & 15, b & 7
        if e == 15 and m == 7:
            v[b] = np.nan
        elif e == 0:
            v[b] = s * m / 8.0 * 2.0 ** -6
        else:
            v[b] = s * (1.0 + m / 8.0) * 2.0 ** (e - 7)
    return v


def e4m3_encode(x: np.ndarray) -> np.ndarray:
    """Round-half-to-even e4m3fn codes of finite values with |x| <= 448 (float64 arithmetic is exact here)."""
    x = np.asarray(x, dtype=np.float64)
    if np.any(~np.isfinite(x)) or np.any(np.abs(x) > E4M3_MAX):
        raise ValueError("e4m3_encode: finite |x| <= 448 only (the MX8 block scale guarantees it)")
    sign = (np.signbit(x)).astype(np.uint8) << 7
    a = np.abs(x)
    code = np.zeros(a.shape, dtype=np.int64)
    sub = a < 2.0 ** -6
    # subnormal range: multiples of 2^-9; a rounded count of 8 is the smallest normal (code 0x08) as it should be
    code[sub] = np.round(a[sub] / 2.0 ** -9).astype(np.int64)
    nrm = ~sub
    if np.any(nrm):
        e = np.floor(np.log2(a[nrm])).astype(np.int64)
        # guard log2 rounding at exact powers of two
        e = np.where(a[nrm] < 2.0 ** e, e - 1, e)
        e = np.where(a[nrm] >= 2.0 ** (e + 1), e + 1, e)
        m = np.round((a[nrm] / 2.0 ** e - 1.0) * 8.0).astype(np.int64)
        carry = m == 8
        e = np.where(carry, e + 1, e)
        m = np.where(carry, 0, m)
        if np.any(e > 8):
            raise ValueError("e4m3_encode: overflow")
        code[nrm] = ((e + 7) << 3) | m
    return (code.astype(np.uint8) | sign)


def block_exponent(amax_bf16_bits: np.ndarray) -> np.ndarray:
    """E for a block whose |x| max has the bf16 bit pattern `amax_bf16_bits` (sign clear)."""
    am = np.asarray(amax_bf16_bits, dtype=np.int64)
    be = am >> 7
    ex = np.where(be > 0, be - 127, -126)
    E = ex - 8 + ((am & 0x7F) > 0x60).astype(np.int64)
    return np.clip(E, -127, 125)


def quantize(x_bf16: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """bf16 rows [rows][K] (as a uint16 bit array, K % 32 == 0) -> (uint8 codes [rows][K], int scale bytes
    [rows][K/32])."""
    bits = np.asarray(x_bf16, dtype=np.uint16)
    rows, K = bits.shape
    if K % 32:
        raise ValueError("K % 32 == 0")
    x = (bits.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    mag = (bits & 0x7FFF).astype(np.int64).reshape(rows, K // 32, 32)
    E = block_exponent(mag.max(axis=2))
    scaled = x.reshape(rows, K // 32, 32) * np.exp2(-E.astype(np.float64))[..., None]
    codes = e4m3_encode(scaled).reshape(rows, K)
    return codes, (E + 127).astype(np.int64)


def dequantize(codes: np.ndarray, scale_bytes: np.ndarray) -> np.ndarray:
    """float64 values of an MX8 operand ([rows][K] codes, [rows][K/32] scale bytes)."""
    v = e4m3_value_table()[np.asarray(codes, dtype=np.int64)]
    return v * np.repeat(np.exp2(np.asarray(scale_bytes, dtype=np.float64) - 127.0), 32, axis=1)[:, :v.shape[1]]


def scale_byte_index(r: np.ndarray, k: np.ndarray, lds: int) -> np.ndarray:
    """Byte offset of the scale of (row r, K value k) in the scale planes (vpf.h "MX8 operands")."""
    r = np.asarray(r, dtype=np.int64)
    k = np.asarray(k, dtype=np.int64)
    return ((k >> 7) * lds + (r >> 6) * 64 + ((k >> 5) & 3) * 16 + (r & 15)) * 4 + ((r >> 4) & 3)


def pack_scales(scale_bytes: np.ndarray, lds: int) -> np.ndarray:
    """[rows][K/32] scale bytes -> int32 [K/128][lds] planes in the device layout."""
    rows, nb = scale_bytes.shape
    out = np.zeros((nb // 4) * lds * 4, dtype=np.uint8)
    r, b = np.meshgrid(np.arange(rows), np.arange(nb), indexing="ij")
    out[scale_byte_index(r, b * 32, lds)] = scale_bytes.astype(np.uint8)
    return out.view(np.int32).reshape(nb // 4, lds)


def gemm(a_codes, a_scales, w_codes, w_scales) -> np.ndarray:
    """value(A) . value(W)^T in float64: what the block-scaled MFMA computes before its fp32 accumulation order."""
    return dequantize(a_codes, a_scales) @ dequantize(w_codes, w_scales).T
