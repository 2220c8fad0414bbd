"""ctypes binding of libvpf.so (the C-ABI in include/vpf.h).

This is the binding a maintainer of the reference would add for its `Tracker` / `ParticleFilter` hot
path (the reference itself has no FFI: README-only, /root/reference/README.md:1-63); INTEGRATION.md
reproduces it. `torch` is imported first so that libvpf's NEEDED `libamdhip64.so.7` resolves to the HIP
runtime PyTorch already loaded (same SONAME) — kernels and torch then share one runtime and torch's
stream handles are valid here.

There is no fallback: if the library is missing or fails to load, every product entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VPF_LIB_PATH") or os.path.join(_HERE, "libvpf.so")   # override: A/B tooling only
CSRC = os.path.join(_HERE, "csrc")

_lock = threading.Lock()
_lib = None

VPF_EPI_BIAS = 0
VPF_EPI_BIAS_GELU = 1
VPF_EPI_BIAS_RESIDUAL = 2
VPF_EPI_PATCH = 3
VPF_EPI_LN = 4
VPF_EPI_LN_GELU = 5

_P, _I64, _I32, _U64, _U32, _F32 = (ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_uint64,
                                    ctypes.c_uint32, ctypes.c_float)

# name -> argtypes (every function returns int, except vpf_version)
SIGNATURES = {
    "vpf_predict": [_P, _I64, _I64, _I64, _U64, _U32, _F32, _F32, _F32, _F32, _F32, _F32, _F32, _P],
    "vpf_crop_patches_bf16": [_P, _I32, _I32, _P, _P, _I64, _I64, _F32, _F32, _I32, _I32, _I32, _P, _P, _P],
    "vpf_crop_patches_f32": [_P, _I32, _I32, _P, _P, _I64, _I64, _F32, _F32, _I32, _I32, _I32, _P, _P, _P],
    "vpf_cls_rows_bf16": [_P, _I64, _I32, _I32, _P, _P, _P, _I32, _P],
    "vpf_cls_rows_f32": [_P, _I64, _I32, _I32, _P, _P, _P],
    "vpf_gemm_bf16": [_P, _I64, _P, _P, _P, _P, _I32, _P, _P, _P, _I64, _I64, _I64, _I64, _I32, _I32, _F32, _P,
                      _P, _I64, _P, _I64, _P],
    "vpf_gemm_mx8": [_P, _I64, _P, _I64, _P, _P, _P, _P, _P, _P, _P, _I64, _P, _I64, _P, _I64, _I64, _I64, _I64,
                     _I32, _I32, _F32, _P, _P],
    "vpf_quantize_mx8": [_P, _I64, _I64, _I64, _I64, _P, _I64, _P, _I64, _P],
    "vpf_gemm_bf16_splitk": [_P, _I64, _P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _I32, _I32, _P, _P, _I64, _P],
    "vpf_gemm_tune": [_I32, _I32],
    "vpf_gemm_f32": [_P, _I64, _P, _P, _P, _P, _I32, _P, _P, _P, _I64, _I64, _I64, _I64, _I32, _P],
    "vpf_row_stats_bf16": [_P, _I64, _I32, _I64, _F32, _P, _P],
    "vpf_stats_combine": [_P, _I32, _I64, _I64, _I32, _F32, _P, _P],
    "vpf_row_stats_f32": [_P, _I64, _I32, _I64, _F32, _P, _P],
    "vpf_layernorm_bf16": [_P, _I64, _I32, _I64, _P, _P, _F32, _P, _I64, _P],
    "vpf_layernorm_f32": [_P, _I64, _I32, _I64, _P, _P, _F32, _P, _I64, _P],
    "vpf_attention_bf16": [_P, _P, _I64, _I32, _I32, _I32, _F32, _I32, _P],
    "vpf_attention_f32": [_P, _P, _I64, _I32, _I32, _I32, _F32, _I32, _P],
    "vpf_attention_bf16_mx8": [_P, _I64, _I32, _I32, _I32, _F32, _P, _I64, _P, _I64, _P],
    "vpf_head_gather_bf16": [_P, _I64, _I32, _I32, _P, _I64, _P],
    "vpf_cls_attn_fold_bf16": [_P, _I64, _I32, _I32, _P, _I64, _F32, _P, _I64, _P, _I64, _P, _F32, _P, _I64, _P],
    "vpf_cls_weight_bf16": [_P, _I64, _I32, _I32, _P, _P, _F32, _P, _F32, _I32, _P, _P, _P, _P],
    "vpf_cls_weight_f32": [_P, _I64, _I32, _I32, _P, _P, _F32, _P, _F32, _I32, _P, _P, _P, _P],
    "vpf_cosine_weight_f32": [_P, _I64, _I32, _P, _F32, _I32, _P, _P, _P],
    "vpf_shard_stats": [_P, _P, _I64, _I64, _P, _P, _P],
    "vpf_resample": [_P, _I64, _I64, _I64, _I64, _I64, _U32, _I32, _I64, _I64, _P, _I64, _P, _P, _I64, _P, _P],
    "vpf_estimate_resample": [_P, _I64, _P, _I64, _I64, _I64, _I64, _U64, _U32, _I64, _I64, _P, _P, _I64, _P, _P,
                              _P],
}


class VPFError(RuntimeError):
    pass


def build(force: bool = False) -> str:
    """Compile libvpf.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    args = ["make", "-s", "-C", CSRC, "-j8"]
    if force:
        subprocess.run(["make", "-s", "-C", CSRC, "clean"], check=True)
    subprocess.run(args, check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    """Load libvpf.so (once). Raises VPFError when it is missing — there is no CPU fallback."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise VPFError(f"libvpf.so not found at {LIB_PATH}; run `python -c 'import __graft_entry__ as g; "
                               f"g.build()'` (or `make -C {CSRC}`)")
            L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            override = os.environ.get("VPF_LIB_PATH") is not None
            for name, argtypes in SIGNATURES.items():
                if override and not hasattr(L, name):
                    continue   # an A/B build (lab / older snapshot) may lack newer entry points; the product never
                fn = getattr(L, name)
                fn.argtypes = argtypes
                fn.restype = ctypes.c_int
            L.vpf_version.argtypes = []
            L.vpf_version.restype = ctypes.c_char_p
            _lib = L
    return _lib


def check(rc: int, name: str) -> None:
    if rc != 0:
        if rc == -1:
            raise VPFError(f"{name}: argument violates the shape contract of include/vpf.h")
        raise VPFError(f"{name}: HIP error {rc}")


def stream_ptr(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)
