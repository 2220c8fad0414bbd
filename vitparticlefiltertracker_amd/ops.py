"""PyTorch-ROCm custom ops `torch.ops.vpf.*` over the libvpf C-ABI.

Every op is registered for the CUDA (= HIP on ROCm) device only: called with CPU tensors it raises, and
if libvpf.so is missing it raises — the product path has no CPU fallback (the CPU restatement lives in
oracle/ and is test infrastructure). Ops write into caller-provided outputs (`Tensor(a!)` out
arguments), so a whole frame can be captured into one HIP graph (vit.py) with every buffer preallocated.
Kernels run on torch's current HIP stream.
"""
from __future__ import annotations

from typing import List, Optional

import torch

from . import _lib
from ._lib import call, ptr, stream_ptr

_BF16 = torch.bfloat16
_F32 = torch.float32


def _chk(cond: bool, msg: str) -> None:
    if not cond:
        raise ValueError(msg)


def _dev(*ts) -> None:
    for t in ts:
        if t is not None:
            _chk(t.is_cuda, "vpf ops run on the GPU only (no CPU fallback); got a CPU tensor")
            _chk(t.is_contiguous(), "vpf ops expect contiguous tensors")


@torch.library.custom_op("vpf::predict_", mutates_args={"particles"}, device_types="cuda")
def predict_(particles: torch.Tensor, global_begin: int, seed: int, frame: int, motion_std: List[float],
             width: float, height: float, scale_range: List[float]) -> None:
    """H1, SPEC S2: in-place random walk on particles float32[3][n]."""
    _dev(particles)
    _chk(particles.dtype == _F32 and particles.dim() == 2 and particles.shape[0] == 3, "particles: f32[3][n]")
    n = particles.shape[1]
    call("vpf_predict", ptr(particles), n, n, global_begin, seed & (2**64 - 1), frame, motion_std[0],
         motion_std[1], motion_std[2], width, height, scale_range[0], scale_range[1], stream_ptr())


def rgba_workspace(frame_hw, device) -> torch.Tensor:
    """Workspace for crop_patches: int32[(H+2)*(W+2)] (the zero-bordered RGBA frame)."""
    H, W = int(frame_hw[0]), int(frame_hw[1])
    return torch.empty((H + 2) * (W + 2), device=device, dtype=torch.int32)


@torch.library.custom_op("vpf::crop_patches", mutates_args={"rgba_ws", "out"}, device_types="cuda")
def crop_patches(frame: torch.Tensor, rgba_ws: torch.Tensor, particles: torch.Tensor, box_wh: List[float],
                 img_size: int, patch: int, norm_ab: List[float], out: torch.Tensor) -> None:
    """H2+H3 A operand, SPEC S3: out[n*g*g][Kp] (bf16 or f32). rgba_ws: rgba_workspace(frame.shape[:2])."""
    _dev(frame, rgba_ws, particles, out)
    _chk(frame.dtype == torch.uint8 and frame.dim() == 3 and frame.shape[2] == 3, "frame: u8[H][W][3]")
    _chk(rgba_ws.dtype == torch.int32 and rgba_ws.is_contiguous()
         and rgba_ws.numel() >= (frame.shape[0] + 2) * (frame.shape[1] + 2), "rgba_ws: int32[(H+2)*(W+2)]")
    _chk(particles.dtype == _F32 and particles.dim() == 2 and particles.shape[0] == 3, "particles: f32[3][n]")
    n = particles.shape[1]
    g = img_size // patch
    kp = out.shape[1]
    _chk(out.dim() == 2 and out.shape[0] == n * g * g, "out: [n*g*g][Kp]")
    ab = (torch.tensor(norm_ab, dtype=torch.float32)).numpy()
    import ctypes
    abp = ab.ctypes.data_as(ctypes.c_void_p)
    name = "vpf_crop_patches_bf16" if out.dtype == _BF16 else "vpf_crop_patches_f32"
    _chk(out.dtype in (_BF16, _F32), "out dtype must be bf16 or f32")
    call(name, ptr(frame), frame.shape[0], frame.shape[1], ptr(rgba_ws), ptr(particles), n, n, box_wh[0], box_wh[1],
         img_size, patch, kp, abp, ptr(out), stream_ptr())


@torch.library.custom_op("vpf::cls_rows_", mutates_args={"tokens"}, device_types="cuda")
def cls_rows_(tokens: torch.Tensor, cls: torch.Tensor, pos: torch.Tensor) -> None:
    """H3: tokens[p][0][:] = cls + pos[0]; tokens [n][N][D]."""
    _dev(tokens, cls, pos)
    n, N, D = tokens.shape
    if tokens.dtype == _BF16:
        call("vpf_cls_rows_bf16", ptr(tokens), n, N, D, ptr(cls), ptr(pos), None, 0, stream_ptr())
    else:
        call("vpf_cls_rows_f32", ptr(tokens), n, N, D, ptr(cls), ptr(pos), stream_ptr())


@torch.library.custom_op("vpf::cls_rows_stats_", mutates_args={"tokens", "stats_out"}, device_types="cuda")
def cls_rows_stats_(tokens: torch.Tensor, cls: torch.Tensor, pos: torch.Tensor, stats_out: torch.Tensor) -> None:
    """cls_rows_ (bf16) that also writes the CLS rows' {sum, sumsq} into the residual-stream statistics planes
    `stats_out` [P][n*N][2] f32 (plane 0; other planes 0), the layout vpf_gemm_bf16 producers write."""
    _dev(tokens, cls, pos, stats_out)
    n, N, D = tokens.shape
    _chk(tokens.dtype == _BF16, "cls_rows_stats_: bf16 tokens")
    _chk(stats_out.dtype == _F32 and stats_out.dim() == 3 and tuple(stats_out.shape[1:]) == (n * N, 2),
         "cls_rows_stats_: stats_out f32[P][n*N][2]")
    call("vpf_cls_rows_bf16", ptr(tokens), n, N, D, ptr(cls), ptr(pos), ptr(stats_out), stats_out.shape[0],
         stream_ptr())


def _rows(t: torch.Tensor, what: str):
    """(rows, row stride) of a 2-D row-major view whose rows may be strided (last dim contiguous)."""
    _chk(t.dim() == 2 and t.stride(1) == 1, f"{what}: expected a 2-D view with unit column stride")
    return t.shape[0], t.stride(0)


def _gemm(a, w, bias, residual, pos, patch_rows, row_stats, colsum, epilogue, out, stats_parts, ln_eps, stats_out,
          q8=None, s8=None):
    _dev(w, bias, pos, row_stats, colsum, stats_out)
    for t in (a, out, residual):
        if t is not None:
            _chk(t.is_cuda, "vpf ops run on the GPU only (no CPU fallback); got a CPU tensor")
    M, lda = _rows(a, "gemm a")
    K = a.shape[1]
    N = w.shape[0]
    _chk(w.shape[1] == K and bias.numel() == N and bias.dtype == _F32, "gemm: shape mismatch")
    _chk(a.dtype == w.dtype == out.dtype, "gemm: a, w, out must share a dtype")
    if epilogue == _lib.VPF_EPI_PATCH:
        _chk(out.is_contiguous() and out.numel() >= (M // patch_rows) * (patch_rows + 1) * N,
             "gemm: patch output too small")
        ldc = N
    else:
        Mo, ldc = _rows(out, "gemm out")
        _chk(Mo == M and out.shape[1] == N, "gemm: output shape")
    if residual is not None:
        _chk(_rows(residual, "gemm residual") == (M, ldc), "gemm: residual must match out's layout")
    if epilogue in (_lib.VPF_EPI_LN, _lib.VPF_EPI_LN_GELU):
        _chk(row_stats is not None and row_stats.numel() >= 2 * M * max(stats_parts, 1) and colsum is not None
             and colsum.numel() == N, "gemm: LN epilogue needs row_stats [max(P,1)][M][2] and colsum[N]")
    if a.dtype == _BF16:
        if stats_out is not None:
            R = (M // patch_rows) * (patch_rows + 1) if epilogue == _lib.VPF_EPI_PATCH else M
            _chk(stats_out.dtype == _F32 and stats_out.numel() >= ((N + 63) // 64) * R * 2,
                 "gemm: stats_out f32[ceil(N/64)][rows][2]")
        ld8, lds = _mx8_out(q8, s8, (M // patch_rows) * (patch_rows + 1) if epilogue == _lib.VPF_EPI_PATCH else M, N)
        call("vpf_gemm_bf16", ptr(a), lda, ptr(w), ptr(bias), ptr(residual), ptr(pos), patch_rows, ptr(row_stats),
             ptr(colsum), ptr(out), ldc, M, N, K, epilogue, stats_parts, ln_eps, ptr(stats_out), ptr(q8), ld8, ptr(s8),
             lds, stream_ptr())
    else:
        _chk(stats_parts == 0 and stats_out is None, "gemm: statistics planes are a bf16-path feature")
        call("vpf_gemm_f32", ptr(a), lda, ptr(w), ptr(bias), ptr(residual), ptr(pos), patch_rows, ptr(row_stats),
             ptr(colsum), ptr(out), ldc, M, N, K, epilogue, stream_ptr())


@torch.library.custom_op("vpf::gemm", mutates_args={"out"}, device_types="cuda")
def gemm(a: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, residual: Optional[torch.Tensor],
         pos: Optional[torch.Tensor], patch_rows: int, row_stats: Optional[torch.Tensor],
         colsum: Optional[torch.Tensor], epilogue: int, out: torch.Tensor, stats_parts: int = 0,
         ln_eps: float = 0.0) -> None:
    """H3/H5/H7/H8: out = epilogue(a[M][K] . w[N][K]^T) (bf16 MFMA or fp32 parity mode by dtype).

    `a`, `out` (and `residual`, which must share `out`'s row stride) are 2-D views whose rows may be strided
    (e.g. the CLS rows of the token tensor). EPI_PATCH takes `out` as the flat token buffer.
    bf16 LN epilogues: `stats_parts` = 0 reads `row_stats` as {mean, rstd} rows (vpf_row_stats); P > 0 reads it
    as P residual-stream statistics planes [P][M][2] of {sum, sumsq} (written by gemm_stats_ / cls_rows_stats_)
    combined with `ln_eps`."""
    _gemm(a, w, bias, residual, pos, patch_rows, row_stats, colsum, epilogue, out, stats_parts, ln_eps, None)


@torch.library.custom_op("vpf::gemm_stats_", mutates_args={"out", "stats_out"}, device_types="cuda")
def gemm_stats_(a: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, residual: Optional[torch.Tensor],
                pos: Optional[torch.Tensor], patch_rows: int, epilogue: int, out: torch.Tensor,
                stats_out: torch.Tensor) -> None:
    """gemm (bf16, EPI_BIAS_RESIDUAL / EPI_PATCH) that also writes the residual-stream statistics planes of its
    output: `stats_out` [ceil(N/64)][rows][2] f32, per row {sum, sumsq} of the stored bf16 values over each
    64-column block (rows = output rows; token rows for EPI_PATCH, whose CLS rows cls_rows_stats_ fills)."""
    _gemm(a, w, bias, residual, pos, patch_rows, None, None, epilogue, out, 0, 0.0, stats_out)


@torch.library.custom_op("vpf::gemm_splitk_", mutates_args={"out", "stats_out", "ws"}, device_types="cuda")
def gemm_splitk_(a: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, residual: Optional[torch.Tensor],
                 row_stats: Optional[torch.Tensor], colsum: Optional[torch.Tensor], epilogue: int, splits: int,
                 out: torch.Tensor, stats_out: Optional[torch.Tensor], ws: torch.Tensor) -> None:
    """Split-K bf16 GEMM (vpf_gemm_bf16_splitk) for few-row GEMMs: `splits` K-chunks into the fp32 workspace `ws`
    (>= splits*M*N), summed in split order, then the epilogue (BIAS, BIAS_GELU, BIAS_RESIDUAL [+ stats_out planes
    [N/64][M][2]], LN / LN_GELU with {mean, rstd} row_stats). `a`, `out`, `residual` may be row-strided views."""
    _dev(w, bias, row_stats, colsum, stats_out, ws)
    for t in (a, out, residual):
        if t is not None:
            _chk(t.is_cuda, "vpf ops run on the GPU only (no CPU fallback); got a CPU tensor")
    M, lda = _rows(a, "gemm_splitk a")
    K, N = a.shape[1], w.shape[0]
    _chk(a.dtype == w.dtype == out.dtype == _BF16, "gemm_splitk: bf16 operands")
    _chk(w.shape[1] == K and bias.numel() == N and bias.dtype == _F32, "gemm_splitk: shape mismatch")
    Mo, ldc = _rows(out, "gemm_splitk out")
    _chk(Mo == M and out.shape[1] == N, "gemm_splitk: output shape")
    if residual is not None:
        _chk(_rows(residual, "gemm_splitk residual") == (M, ldc), "gemm_splitk: residual must match out's layout")
    if epilogue in (_lib.VPF_EPI_LN, _lib.VPF_EPI_LN_GELU):
        _chk(row_stats is not None and row_stats.numel() >= 2 * M and colsum is not None and colsum.numel() == N,
             "gemm_splitk: LN epilogue needs {mean, rstd} row_stats [M][2] and colsum[N]")
    if stats_out is not None:
        _chk(stats_out.dtype == _F32 and stats_out.numel() >= (N // 64) * M * 2, "gemm_splitk: stats_out [N/64][M][2]")
    _chk(ws.dtype == _F32 and ws.numel() >= splits * M * N, "gemm_splitk: workspace f32[splits*M*N]")
    call("vpf_gemm_bf16_splitk", ptr(a), lda, ptr(w), ptr(bias), ptr(residual), ptr(row_stats), ptr(colsum), ptr(out),
         ldc, M, N, K, epilogue, splits, ptr(stats_out), ptr(ws), ws.numel(), stream_ptr())


# ---------------------------------------------------------------------------------------------- MX8 (fp8 path)
# An MX8 tensor is a pair (q, s): q uint8[rows][K] (e4m3fn codes; a row-strided view is allowed) and s int32
# [K/128][lds] scale planes (e8m0 bytes in 64-row bricks, vpf.h "MX8 operands"), lds = rows rounded up to 64.

def mx8_empty(rows: int, K: int, device, lds_rows: Optional[int] = None):
    """Allocate an MX8 operand for `rows` rows of K values (scale planes for lds_rows >= rows rows)."""
    _chk(K % 128 == 0, "mx8: K % 128 == 0")
    lds = ((max(rows, lds_rows or 0) + 63) // 64) * 64
    return (torch.empty(rows, K, device=device, dtype=torch.uint8),
            torch.empty(K // 128, lds, device=device, dtype=torch.int32))


def _mx8_in(q, s, what):
    _chk(q is not None and s is not None and q.is_cuda and s.is_cuda, f"{what}: MX8 operand on the GPU")
    _chk(q.dtype == torch.uint8 and s.dtype == torch.int32 and s.dim() == 2 and s.is_contiguous(),
         f"{what}: MX8 operand = (uint8[rows][K], int32[K/128][lds])")
    rows, ld = _rows(q, what)
    _chk(s.shape[0] == q.shape[1] // 128 and s.shape[1] >= rows and s.shape[1] % 64 == 0, f"{what}: scale planes")
    return rows, ld, s.shape[1]


def _mx8_out(q8, s8, rows, N):
    if q8 is None:
        _chk(s8 is None, "fp8 output: pass both q8 and s8")
        return 0, 0
    _chk(s8 is not None and q8.is_cuda and s8.is_cuda and q8.dtype == torch.uint8 and s8.dtype == torch.int32,
         "fp8 output: (uint8, int32) MX8 pair")
    qr, ld8 = _rows(q8, "fp8 output")
    _chk(qr >= rows and q8.shape[1] >= N and s8.is_contiguous() and s8.shape[0] == N // 128
         and s8.shape[1] >= rows and s8.shape[1] % 64 == 0, "fp8 output: shape / scale planes")
    return ld8, s8.shape[1]


@torch.library.custom_op("vpf::gemm_q8_", mutates_args={"out", "stats_out", "q8", "s8"}, device_types="cuda")
def gemm_q8_(a: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, residual: Optional[torch.Tensor],
             pos: Optional[torch.Tensor], patch_rows: int, epilogue: int, out: torch.Tensor, stats_out: torch.Tensor,
             q8: torch.Tensor, s8: torch.Tensor) -> None:
    """gemm_stats_ (bf16 residual-stream producer: EPI_BIAS_RESIDUAL / EPI_PATCH) that also writes an MX8 copy
    (q8, s8) of its bf16 output — the A operand of the fp8 path's following gemm_mx8."""
    _gemm(a, w, bias, residual, pos, patch_rows, None, None, epilogue, out, 0, 0.0, stats_out, q8, s8)


def _gemm_mx8(a8, as8, w8, ws8, bias, residual, row_stats, colsum, epilogue, out, q8, s8, stats_parts, ln_eps,
              stats_out):
    _dev(bias, row_stats, colsum, stats_out, w8, ws8)
    M, lda, lds_a = _mx8_in(a8, as8, "gemm_mx8 a")
    N, K = w8.shape
    _chk(a8.shape[1] == K and ws8.shape == (K // 128, N) and w8.dtype == torch.uint8 and ws8.dtype == torch.int32,
         "gemm_mx8: w = (uint8[N][K], int32[K/128][N])")
    _chk(bias.numel() == N and bias.dtype == _F32, "gemm_mx8: bias f32[N]")
    ldc = 0
    if out is not None:
        Mo, ldc = _rows(out, "gemm_mx8 out")
        _chk(out.is_cuda and out.dtype == _BF16 and Mo == M and out.shape[1] == N, "gemm_mx8: out bf16[M][N]")
    if residual is not None:
        _chk(_rows(residual, "gemm_mx8 residual") == (M, ldc), "gemm_mx8: residual must match out's layout")
    if epilogue in (_lib.VPF_EPI_LN, _lib.VPF_EPI_LN_GELU):
        _chk(row_stats is not None and row_stats.numel() >= 2 * M * max(stats_parts, 1) and colsum is not None
             and colsum.numel() == N, "gemm_mx8: LN epilogue needs row_stats [max(P,1)][M][2] and colsum[N]")
    if stats_out is not None:
        _chk(stats_out.dtype == _F32 and stats_out.numel() >= ((N + 63) // 64) * M * 2,
             "gemm_mx8: stats_out f32[ceil(N/64)][M][2]")
    ld8, lds = _mx8_out(q8, s8, M, N)
    call("vpf_gemm_mx8", ptr(a8), lda, ptr(as8), lds_a, ptr(w8), ptr(ws8), ptr(bias), ptr(residual), ptr(row_stats),
         ptr(colsum), ptr(out), ldc, ptr(q8), ld8, ptr(s8), lds, M, N, K, epilogue, stats_parts, ln_eps, ptr(stats_out),
         stream_ptr())


@torch.library.custom_op("vpf::gemm_mx8", mutates_args={"out"}, device_types="cuda")
def gemm_mx8(a8: torch.Tensor, as8: torch.Tensor, w8: torch.Tensor, ws8: torch.Tensor, bias: torch.Tensor,
             residual: Optional[torch.Tensor], row_stats: Optional[torch.Tensor], colsum: Optional[torch.Tensor],
             epilogue: int, out: torch.Tensor, stats_parts: int = 0, ln_eps: float = 0.0) -> None:
    """fp8 path (configs[4]): out(bf16) = epilogue(value(a8, as8) . value(w8, ws8)^T) on block-scaled MFMA.
    Epilogues and LN statistics as `gemm` (colsum = row sums of value(w8); stats_parts <= 13)."""
    _gemm_mx8(a8, as8, w8, ws8, bias, residual, row_stats, colsum, epilogue, out, None, None, stats_parts, ln_eps,
              None)


@torch.library.custom_op("vpf::gemm_mx8_q8_", mutates_args={"q8", "s8"}, device_types="cuda")
def gemm_mx8_q8_(a8: torch.Tensor, as8: torch.Tensor, w8: torch.Tensor, ws8: torch.Tensor, bias: torch.Tensor,
                 row_stats: Optional[torch.Tensor], colsum: Optional[torch.Tensor], epilogue: int, q8: torch.Tensor,
                 s8: torch.Tensor, stats_parts: int = 0, ln_eps: float = 0.0) -> None:
    """gemm_mx8 whose output is MX8 only (q8, s8): the bf16 epilogue values quantised in the epilogue (FC1 ->
    the A operand of FC2); no bf16 output is written."""
    _gemm_mx8(a8, as8, w8, ws8, bias, None, row_stats, colsum, epilogue, None, q8, s8, stats_parts, ln_eps, None)


@torch.library.custom_op("vpf::gemm_mx8_res_", mutates_args={"out", "stats_out", "q8", "s8"}, device_types="cuda")
def gemm_mx8_res_(a8: torch.Tensor, as8: torch.Tensor, w8: torch.Tensor, ws8: torch.Tensor, bias: torch.Tensor,
                  out: torch.Tensor, stats_out: torch.Tensor, q8: torch.Tensor, s8: torch.Tensor) -> None:
    """Residual-stream producer on the fp8 path (FC2): out += value(a8) value(w8)^T + bias in place (bf16), plus
    its statistics planes and its MX8 copy (q8, s8) for the next block's LN-folded gemm_mx8."""
    _gemm_mx8(a8, as8, w8, ws8, bias, out, None, None, _lib.VPF_EPI_BIAS_RESIDUAL, out, q8, s8, 0, 0.0, stats_out)


@torch.library.custom_op("vpf::quantize_mx8_", mutates_args={"q8", "s8"}, device_types="cuda")
def quantize_mx8_(x: torch.Tensor, out_stride: int, q8: torch.Tensor, s8: torch.Tensor) -> None:
    """MX8 quantisation of bf16 rows: row r of the (row-strided) view x -> row r*out_stride of (q8, s8)."""
    _chk(x.is_cuda and x.dtype == _BF16, "quantize_mx8_: bf16 rows on the GPU")
    rows, ldx = _rows(x, "quantize_mx8_ x")
    K = x.shape[1]
    _chk(q8.is_cuda and s8.is_cuda and q8.dtype == torch.uint8 and s8.dtype == torch.int32 and s8.is_contiguous(),
         "quantize_mx8_: (uint8, int32) output pair")
    qr, ld8 = _rows(q8, "quantize_mx8_ q8")
    _chk(qr >= (rows - 1) * out_stride + 1 and q8.shape[1] >= K and s8.shape[0] == K // 128,
         "quantize_mx8_: output shape")
    call("vpf_quantize_mx8", ptr(x), ldx, rows, K, out_stride, ptr(q8), ld8, ptr(s8), s8.shape[1], stream_ptr())


_E4M3 = None


def e4m3_table(device) -> torch.Tensor:
    """float32[256]: the OCP e4m3fn value of every byte (NaN for 0x7f / 0xff)."""
    global _E4M3
    if _E4M3 is None:
        v = []
        for b in range(256):
            sgn = -1.0 if b & 0x80 else 1.0
            e, m = (b >> 3) & 15, b & 7
            if e == 15 and m == 7:
                v.append(float("nan"))
            elif e == 0:
                v.append(sgn * m / 8.0 * 2.0 ** -6)
            else:
                v.append(sgn * (1.0 + m / 8.0) * 2.0 ** (e - 7))
        _E4M3 = torch.tensor(v, dtype=torch.float32)
    return _E4M3.to(device)


def mx8_scale_bytes(s8: torch.Tensor, rows: int) -> torch.Tensor:
    """int32[rows][K/32]: the e8m0 scale byte of every (row, 32-value block) of an MX8 operand's planes."""
    T, lds = s8.shape
    b = s8.contiguous().view(torch.uint8).view(T, lds * 4)
    r = torch.arange(rows, device=s8.device)
    kb = torch.arange(4, device=s8.device)
    idx = (((r >> 6) * 64 + (r & 15))[:, None] + kb[None, :] * 16) * 4 + ((r >> 4) & 3)[:, None]   # [rows][4]
    out = b[:, idx.reshape(-1)].view(T, rows, 4).permute(1, 0, 2).reshape(rows, T * 4)
    return out.to(torch.int32)


def mx8_dequantize(q8: torch.Tensor, s8: torch.Tensor) -> torch.Tensor:
    """float32[rows][K] values of an MX8 operand (setup-time use: the LN-fold colsum of fp8 weights; tests)."""
    rows, K = q8.shape
    vals = e4m3_table(q8.device)[q8.long()]
    sc = torch.exp2(mx8_scale_bytes(s8, rows).float() - 127.0)
    return vals * sc.repeat_interleave(32, dim=1)[:, :K]


@torch.library.custom_op("vpf::row_stats", mutates_args={"out"}, device_types="cuda")
def row_stats(x: torch.Tensor, eps: float, out: torch.Tensor) -> None:
    """H4 (folded): out[r] = (mean, rstd) of row r of the 2-D (row-strided) view x."""
    _dev(out)
    _chk(x.is_cuda, "vpf ops run on the GPU only")
    rows, xs = _rows(x, "row_stats x")
    _chk(out.dtype == _F32 and out.numel() >= 2 * rows, "row_stats: out f32[rows][2]")
    name = "vpf_row_stats_bf16" if x.dtype == _BF16 else "vpf_row_stats_f32"
    call(name, ptr(x), rows, x.shape[1], xs, eps, ptr(out), stream_ptr())


@torch.library.custom_op("vpf::stats_combine_", mutates_args={"out"}, device_types="cuda")
def stats_combine_(planes: torch.Tensor, D: int, eps: float, out: torch.Tensor) -> None:
    """H4 (folded): out[r] = (mean, rstd) of row r from the statistics planes f32[P][rows][2] (a producer GEMM's
    stats_out view) over a row length D (vpf_stats_combine; bit-identical to the consuming GEMM's own combine)."""
    _dev(planes, out)
    _chk(planes.dtype == _F32 and planes.dim() == 3 and planes.shape[2] == 2 and planes.stride(2) == 1
         and planes.stride(1) == 2, "stats_combine_: planes f32[P][rows][2]")
    rows = planes.shape[1]
    _chk(out.dtype == _F32 and out.is_contiguous() and out.numel() >= 2 * rows, "stats_combine_: out f32[rows][2]")
    call("vpf_stats_combine", ptr(planes), planes.shape[0], planes.stride(0) // 2, rows, D, eps, ptr(out),
         stream_ptr())


@torch.library.custom_op("vpf::layernorm", mutates_args={"out"}, device_types="cuda")
def layernorm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float, out: torch.Tensor) -> None:
    """H4: row LayerNorm over the last dim of 2-D (row-strided) views x -> out."""
    _dev(gamma, beta)
    _chk(x.is_cuda and out.is_cuda, "vpf ops run on the GPU only")
    rows, xs = _rows(x, "layernorm x")
    ro, ys = _rows(out, "layernorm out")
    _chk(ro == rows and out.shape[1] == x.shape[1], "layernorm: shape")
    name = "vpf_layernorm_bf16" if x.dtype == _BF16 else "vpf_layernorm_f32"
    call(name, ptr(x), rows, x.shape[1], xs, ptr(gamma), ptr(beta), eps, ptr(out), ys, stream_ptr())


@torch.library.custom_op("vpf::attention", mutates_args={"out"}, device_types="cuda")
def attention(qkv: torch.Tensor, heads: int, q_rows: int, out: torch.Tensor) -> None:
    """H6: qkv [B][N][3D] -> out [B][N][D]; only the first q_rows queries of each particle."""
    _dev(qkv, out)
    B, N, D3 = qkv.shape
    D = D3 // 3
    hd = D // heads
    name = "vpf_attention_bf16" if qkv.dtype == _BF16 else "vpf_attention_f32"
    call(name, ptr(qkv), ptr(out), B, N, heads, hd, hd ** -0.5, q_rows, stream_ptr())


@torch.library.custom_op("vpf::attention_q8_", mutates_args={"q8", "s8"}, device_types="cuda")
def attention_q8_(qkv: torch.Tensor, heads: int, q8: torch.Tensor, s8: torch.Tensor) -> None:
    """H6 on the fp8 path: every query row (N <= 256), output written as MX8 (q8, s8) — the proj GEMM's A
    operand — instead of bf16."""
    _dev(qkv, s8)
    _chk(qkv.dtype == _BF16 and q8.is_cuda and q8.dtype == torch.uint8 and s8.dtype == torch.int32,
         "attention_q8_: bf16 qkv, MX8 (uint8, int32) output")
    B, N, D3 = qkv.shape
    D = D3 // 3
    rows, ld8 = _rows(q8, "attention_q8_ q8")
    _chk(rows >= B * N and q8.shape[1] >= D and s8.shape[0] == D // 128, "attention_q8_: output shape")
    call("vpf_attention_bf16_mx8", ptr(qkv), B, N, heads, D // heads, (D // heads) ** -0.5, ptr(q8), ld8, ptr(s8),
         s8.shape[1], stream_ptr())


@torch.library.custom_op("vpf::cls_attn_fold_", mutates_args={"out"}, device_types="cuda")
def cls_attn_fold_(tokens: torch.Tensor, planes: torch.Tensor, eps: float, G: torch.Tensor, q: torch.Tensor,
                   bk: torch.Tensor, heads: int, out: torch.Tensor) -> None:
    """H6 for the last block's CLS query, K / V never formed (LN-folded bf16): tokens [n][N][D] with statistics
    planes [D/64][n*N][2]; G [n][H*D] (W'_k,h^T q_h), q the CLS queries [n][D] (row-strided), bk = b'_k;
    out [n][H*D] = per head sum_j p_hj LNraw_j (vpf_cls_attn_fold_bf16)."""
    _dev(tokens, planes, G, bk, out)
    _chk(q.is_cuda and tokens.dtype == _BF16 and G.dtype == _BF16 and q.dtype == _BF16 and out.dtype == _BF16,
         "cls_attn_fold_: bf16 tokens / G / q / out")
    n, N, D = tokens.shape
    _chk(tokens.is_contiguous() and D == 64 * heads, "cls_attn_fold_: contiguous tokens, head dim 64")
    _chk(planes.dtype == _F32 and planes.dim() == 3 and planes.shape[0] == heads and planes.shape[1] >= n * N
         and planes.stride(2) == 1 and planes.stride(1) == 2, "cls_attn_fold_: planes f32[D/64][n*N][2]")
    _chk(bk.dtype == _F32 and bk.numel() >= D and bk.is_contiguous(), "cls_attn_fold_: bk f32[D]")
    rg, ldg = _rows(G, "cls_attn_fold_ G")
    rq, ldq = _rows(q, "cls_attn_fold_ q")
    ro, ldo = _rows(out, "cls_attn_fold_ out")
    _chk(rg == n and rq == n and ro == n and G.shape[1] == heads * D and q.shape[1] == D and out.shape[1] == heads * D,
         "cls_attn_fold_: shapes")
    call("vpf_cls_attn_fold_bf16", ptr(tokens), n, N, heads, ptr(planes), planes.stride(0) // 2, eps, ptr(G), ldg,
         ptr(q), ldq, ptr(bk), 64 ** -0.5, ptr(out), ldo, stream_ptr())


@torch.library.custom_op("vpf::head_gather_", mutates_args={"out"}, device_types="cuda")
def head_gather_(Y: torch.Tensor, heads: int, out: torch.Tensor) -> None:
    """out[p][h*hd + d] = Y[p*heads + h][h*hd + d]: the diagonal blocks of a per-(particle, head) projection
    (vpf_head_gather_bf16). Y bf16 [n*heads][D] contiguous, out [n][D] row-strided."""
    _dev(Y)
    _chk(out.is_cuda and Y.dtype == _BF16 and out.dtype == _BF16, "head_gather_: bf16 Y / out")
    R, D = Y.shape
    n, ldo = _rows(out, "head_gather_ out")
    _chk(R == n * heads and out.shape[1] == D and D % heads == 0, "head_gather_: shapes")
    call("vpf_head_gather_bf16", ptr(Y), n, heads, D // heads, ptr(out), ldo, stream_ptr())


@torch.library.custom_op("vpf::cls_weight", mutates_args={"Q", "feat", "sim"}, device_types="cuda")
def cls_weight(tokens: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float, tmpl: torch.Tensor,
               lam: float, bits: int, Q: torch.Tensor, feat: Optional[torch.Tensor],
               sim: Optional[torch.Tensor]) -> None:
    """H9+H10: final LN of CLS rows -> cosine with template -> Q = floor(exp(lam(sim-1)) 2^bits)."""
    _dev(tokens, gamma, beta, tmpl, Q, feat, sim)
    n, N, D = tokens.shape
    _chk(Q.dtype == torch.int64 and Q.numel() == n, "Q: int64[n]")
    name = "vpf_cls_weight_bf16" if tokens.dtype == _BF16 else "vpf_cls_weight_f32"
    call(name, ptr(tokens), n, N, D, ptr(gamma), ptr(beta), eps, ptr(tmpl), lam, bits, ptr(feat), ptr(sim),
         ptr(Q), stream_ptr())


@torch.library.custom_op("vpf::cosine_weight", mutates_args={"Q", "sim"}, device_types="cuda")
def cosine_weight(feat: torch.Tensor, tmpl: torch.Tensor, lam: float, bits: int, Q: torch.Tensor,
                  sim: Optional[torch.Tensor]) -> None:
    """H10 alone: Q from explicit fp32 features [n][D] and a unit template (optionally the fp32 cosines)."""
    _dev(feat, tmpl, Q, sim)
    n, D = feat.shape
    _chk(feat.dtype == _F32 and Q.dtype == torch.int64 and Q.numel() == n, "cosine_weight: f32[n][D] -> int64[n]")
    _chk(sim is None or (sim.dtype == _F32 and sim.numel() == n), "cosine_weight: sim f32[n]")
    call("vpf_cosine_weight_f32", ptr(feat), n, D, ptr(tmpl), lam, bits, ptr(sim), ptr(Q), stream_ptr())


@torch.library.custom_op("vpf::shard_stats", mutates_args={"out_T", "out_sums"}, device_types="cuda")
def shard_stats(Q: torch.Tensor, particles: torch.Tensor, out_T: torch.Tensor, out_sums: torch.Tensor) -> None:
    """H11: out_T int64[1] = sum Q, out_sums f64[3] = sum Q*(x, y, s)."""
    _dev(Q, particles, out_T, out_sums)
    n = Q.numel()
    call("vpf_shard_stats", ptr(Q), ptr(particles), particles.shape[1], n, ptr(out_T), ptr(out_sums), stream_ptr())


@torch.library.custom_op("vpf::resample", mutates_args={"anc", "states", "cdf_ws"}, device_types="cuda")
def resample(Q: torch.Tensor, global_begin: int, offset: int, total: int, P: int, U: int, uniform: bool,
             slot_begin: int, slot_end: int, particles: torch.Tensor, anc: torch.Tensor, states: torch.Tensor,
             cdf_ws: torch.Tensor) -> None:
    """H12: ancestors + states of slots [slot_begin, slot_end) whose positions fall in this shard."""
    _dev(Q, particles, anc, states, cdf_ws)
    n_local = Q.numel()
    call("vpf_resample", ptr(Q), n_local, global_begin, offset, total, P, U, int(uniform), slot_begin, slot_end,
         ptr(particles), particles.shape[1], ptr(anc), ptr(states), states.shape[1], ptr(cdf_ws), stream_ptr())


@torch.library.custom_op("vpf::estimate_resample", mutates_args={"anc", "states", "cdf_ws", "stats_out"},
                         device_types="cuda")
def estimate_resample(Q: torch.Tensor, q_stride: int, particles: torch.Tensor, ld: int, p_stride: int, n_shard: int,
                      P: int, seed: int, frame: int, slot_begin: int, slot_end: int, anc: torch.Tensor,
                      states: torch.Tensor, cdf_ws: torch.Tensor, stats_out: torch.Tensor) -> None:
    """H11 + H12 over the global particle set (vpf_estimate_resample): Q int64 / particles f32 are flat views in the
    shard layout (shard r's Q at r*q_stride, its x row at r*p_stride, y / s at + ld / + 2 ld); stats_out int64[4]."""
    _dev(Q, particles, anc, states, cdf_ws, stats_out)
    G = P // n_shard if n_shard > 0 else 0
    _chk(Q.dtype == torch.int64 and particles.dtype == _F32, "estimate_resample: Q int64, particles f32")
    _chk(G >= 1 and G * n_shard == P, "estimate_resample: P must be a multiple of n_shard")
    _chk(Q.numel() >= (G - 1) * q_stride + n_shard, "estimate_resample: Q view too short for the shard layout")
    _chk(particles.numel() >= (G - 1) * p_stride + 2 * ld + n_shard,
         "estimate_resample: particle view too short for the shard layout")
    cnt = slot_end - slot_begin
    _chk(anc.dtype == torch.int32 and anc.numel() >= cnt, "estimate_resample: anc int32[>= slots]")
    _chk(states.dtype == _F32 and states.dim() == 2 and states.shape[0] == 3 and states.shape[1] >= cnt,
         "estimate_resample: states f32[3][>= slots]")
    _chk(cdf_ws.dtype == torch.int64 and cdf_ws.numel() >= P, "estimate_resample: cdf_ws int64[P]")
    _chk(stats_out.dtype == torch.int64 and stats_out.numel() >= 4, "estimate_resample: stats_out int64[4]")
    call("vpf_estimate_resample", ptr(Q), q_stride, ptr(particles), ld, p_stride, n_shard, P, seed & (2**64 - 1),
         frame & 0xFFFFFFFF, slot_begin, slot_end, ptr(anc), ptr(states), states.shape[1], ptr(cdf_ws),
         ptr(stats_out), stream_ptr())
