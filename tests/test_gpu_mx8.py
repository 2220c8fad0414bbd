"""GPU (MI355X): the MX-fp8 path (BASELINE.json configs[4]) — quantiser, block-scaled GEMM
and the fp8 copies written by GEMM epilogues — through the product ops / C-ABI.

References: quantisation is bit-exact against the CPU oracle oracle/mx8.py (the rule in include/vpf.h "MX8
operands": smallest block exponent with amax * 2^-E <= 448, RNE to e4m3fn; pinned by tests/test_oracle_mx8.py);
GEMMs against float64 products of the dequantised operands (so the tolerance covers only fp32 accumulation order
and the final bf16 rounding); every fp8 copy written by an epilogue must equal vpf_quantize_mx8 of the bf16
values the same epilogue stored, bit for bit."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as Fn

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded():
    from vitparticlefiltertracker_amd import _lib, ops  # noqa: F401
    assert b"gfx950" in _lib.lib().vpf_version()


def vpf():
    return torch.ops.vpf


def ops():
    from vitparticlefiltertracker_amd import ops as o
    return o


def E():
    from vitparticlefiltertracker_amd import _lib
    return _lib


def ref_quant(x: torch.Tensor):
    """The oracle's MX8 rule (oracle/mx8.py, pinned by tests/test_oracle_mx8.py): (uint8[rows][K] codes,
    int32[rows][K/32] scale bytes)."""
    from oracle import mx8 as omx8
    bits = x.contiguous().cpu().view(torch.int16).numpy().view(np.uint16)
    codes, sc = omx8.quantize(bits)
    return torch.from_numpy(codes), torch.from_numpy(sc.astype(np.int32))


def quant(x: torch.Tensor):
    q, s = ops().mx8_empty(x.shape[0], x.shape[1], DEV)
    vpf().quantize_mx8_(x, 1, q, s)
    return q, s


def special_rows(K):
    """Rows exercising the block-exponent edges: zeros, subnormal bf16, mantissa 1.75 vs 1.7578 at the top,
    huge / tiny magnitudes, mixed signs."""
    rows = []
    z = torch.zeros(K)
    rows.append(z.clone())
    r = torch.zeros(K); r[::7] = 1e-39; rows.append(r)                     # bf16 subnormals
    for top in (1.75, 1.7578125, 1.0, 1.9921875):
        r = torch.linspace(-1, 1, K) * 0.3; r[5::32] = top * 2.0 ** 10; rows.append(r)
    rows.append(torch.linspace(-3e30, 3e30, K))
    rows.append(torch.linspace(-3e-30, 3e-30, K))
    return torch.stack(rows).to(torch.bfloat16)


@pytest.mark.parametrize("rows,K", [(1, 128), (77, 256), (300, 768), (64, 3072)])
def test_quantize_bit_exact(rows, K):
    g = torch.Generator().manual_seed(rows * K)
    x = (torch.randn(rows, K, generator=g) * torch.exp2(torch.randint(-20, 20, (rows, 1), generator=g).float()))
    x = torch.cat([x.to(torch.bfloat16), special_rows(K)])
    xd = x.to(DEV)
    q, s = quant(xd)
    rq, rs = ref_quant(x)
    assert torch.equal(q.cpu(), rq), f"{(q.cpu() != rq).sum().item()} element codes differ"
    assert torch.equal(ops().mx8_scale_bytes(s, x.shape[0]).cpu(), rs)
    # dequantised values are within half an e4m3 ulp (2^-4 relative) of the input, or exactly 0 below range
    deq = ops().mx8_dequantize(q, s).cpu()
    xf = x.float()
    ok = (deq - xf).abs() <= xf.abs() * 2.0 ** -4 + torch.exp2(rs.float() - 127 - 9).repeat_interleave(32, 1)
    assert bool(ok.all())


def test_quantize_strided_rows():
    """out_stride > 1 (the CLS rows of a token tensor) and a row-strided source view."""
    n, N, D = 9, 5, 256
    tok = (torch.randn(n, N, D, device=DEV)).to(torch.bfloat16)
    cls = tok.view(n, N * D)[:, :D]
    q, s = ops().mx8_empty(n * N, D, DEV)
    q.zero_(); s.zero_()
    vpf().quantize_mx8_(cls, N, q, s)
    rq, rs = ref_quant(cls.contiguous())
    assert torch.equal(q[::N].cpu(), rq)
    assert torch.equal(ops().mx8_scale_bytes(s, n * N)[::N].cpu(), rs)


def _weights(N, K, seed):
    g = torch.Generator().manual_seed(seed)
    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(torch.bfloat16).to(DEV)
    q, s = ops().mx8_empty(N, K, DEV)
    vpf().quantize_mx8_(w, 1, q, s)
    assert s.shape[1] == N
    return q, s, ops().mx8_dequantize(q, s).double()


def _acts(M, K, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(M, K, generator=g) * scale + 0.2).to(torch.bfloat16).to(DEV)
    q, s = quant(x)
    return x, q, s, ops().mx8_dequantize(q, s).double()


def _check(out, ref, lin, A, Wd, extra=0.0):
    """|out - ref| within: the bf16 rounding of the stored value (2^-8 relative: half an ulp, with margin), the
    bf16 rounding of the GEMM value before a residual add (2^-8 |lin|), the block-scaled MFMA's accumulation
    (measured ~1e-5 of sum |a w|; bound 2^-13), and `extra` (the GELU approximation, 2.7e-4)."""
    mag = A.abs() @ Wd.abs().t()
    bound = 2 ** -8 * (ref.abs() + lin.abs()) + 2 ** -13 * mag + extra + 1e-6
    bad = (out.double() - ref).abs() > bound
    assert not bool(bad.any()), f"{int(bad.sum())} of {bad.numel()} outside the bound; worst excess " \
        f"{((out.double() - ref).abs() - bound).max().item():.3g}"


def gelu(x):
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))


@pytest.mark.parametrize("M,N,K", [(777, 256, 128), (300, 768, 768), (1024, 384, 3072), (5, 128, 256)])
@pytest.mark.parametrize("epi", ["bias", "gelu", "res"])
def test_gemm_mx8_plain_epilogues(M, N, K, epi):
    _, a8, as8, A = _acts(M, K, M + K)
    w8, ws8, Wd = _weights(N, K, N + K)
    bias = torch.randn(N, device=DEV) * 0.1
    lin = A @ Wd.t() + bias.double()
    code = {"bias": E().VPF_EPI_BIAS, "gelu": E().VPF_EPI_BIAS_GELU, "res": E().VPF_EPI_BIAS_RESIDUAL}[epi]
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    res = None
    if epi == "res":
        out = (torch.randn(M, N, device=DEV)).to(torch.bfloat16)
        res = out
        ref = out.double() + lin
    else:
        ref = gelu(lin) if epi == "gelu" else lin
    vpf().gemm_mx8(a8, as8, w8, ws8, bias, res, None, None, code, out)
    _check(out, ref, lin, A, Wd, 5e-4 if epi == "gelu" else 0.0)


@pytest.mark.parametrize("M,K,N", [(777, 768, 2304), (513, 256, 384)])
@pytest.mark.parametrize("gelu_epi", [False, True])
@pytest.mark.parametrize("planes", [False, True])
def test_gemm_mx8_layernorm_fold(M, K, N, gelu_epi, planes):
    """LN-folded MX8 GEMM on the raw residual stream: A = MX8(h), W' = MX8(W diag(gamma)), colsum of value(W')."""
    h, a8, as8, A = _acts(M, K, 7 * M + K, scale=0.8)
    g = torch.Generator().manual_seed(N)
    gamma = 1 + 0.2 * torch.randn(K, generator=g)
    beta = 0.1 * torch.randn(K, generator=g)
    W = torch.randn(N, K, generator=g) / math.sqrt(K)
    b = 0.1 * torch.randn(N, generator=g)
    Wg = (W * gamma).to(torch.bfloat16).to(DEV)
    w8, ws8 = ops().mx8_empty(N, K, DEV)
    vpf().quantize_mx8_(Wg, 1, w8, ws8)
    Wd = ops().mx8_dequantize(w8, ws8)
    colsum = Wd.sum(1).float().contiguous()
    bias = (b + W @ beta).to(DEV)
    eps = 1e-6
    hd = h.double()
    if planes:
        P = K // 64
        st = torch.stack([torch.stack([hd[:, 64 * t: 64 * (t + 1)].sum(1), (hd[:, 64 * t: 64 * (t + 1)] ** 2).sum(1)], 1)
                          for t in range(P)]).float().contiguous()
    else:
        P = 0
        st = torch.empty(M, 2, device=DEV)
        vpf().row_stats(h, eps, st)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    code = E().VPF_EPI_LN_GELU if gelu_epi else E().VPF_EPI_LN
    vpf().gemm_mx8(a8, as8, w8, ws8, bias, None, st, colsum, code, out, P, eps)
    mean = hd.mean(1, keepdim=True)
    rstd = 1.0 / torch.sqrt(hd.var(1, unbiased=False, keepdim=True) + eps)
    # the fold's exact algebra on the quantised operands: rstd (value(A) W'^T - mean colsum) + b'
    lin = rstd * (A @ Wd.double().t() - mean * colsum.double()) + bias.double()
    ref = gelu(lin) if gelu_epi else lin
    torch.testing.assert_close(out.double(), ref, rtol=2 ** -8, atol=2e-3)
    # and against LayerNorm -> GEMM in float64 on the unquantised operands: the fp8 error itself (reported bound)
    full = Fn.layer_norm(hd, (K,), gamma.double().to(DEV), beta.double().to(DEV), eps) @ W.double().to(DEV).t() \
        + b.double().to(DEV)
    full = gelu(full) if gelu_epi else full
    rel = ((out.double() - full).norm() / full.norm()).item()
    assert rel < 0.06, rel


def test_gemm_mx8_q8_output_matches_quantizer():
    """FC1-style: the fp8-only output of gemm_mx8_q8_ == quantize_mx8(bf16 output of the same GEMM)."""
    M, K, N = 777, 768, 3072
    _, a8, as8, _ = _acts(M, K, 3)
    w8, ws8, _ = _weights(N, K, 4)
    bias = torch.randn(N, device=DEV) * 0.1
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    st = torch.stack([torch.rand(M, device=DEV) * 0.2 - 0.1, torch.rand(M, device=DEV) + 0.5], 1).contiguous()
    colsum = torch.randn(N, device=DEV)
    LNG = E().VPF_EPI_LN_GELU
    vpf().gemm_mx8(a8, as8, w8, ws8, bias, None, st, colsum, LNG, out)
    q, s = ops().mx8_empty(M, N, DEV)
    vpf().gemm_mx8_q8_(a8, as8, w8, ws8, bias, st, colsum, LNG, q, s)
    rq, rs = quant(out)
    assert torch.equal(q, rq)
    assert torch.equal(ops().mx8_scale_bytes(s, M), ops().mx8_scale_bytes(rs, M))


def _planes_ref(y, P):
    yd = y.double()
    return torch.stack([torch.stack([yd[:, 64 * t: 64 * (t + 1)].sum(1), (yd[:, 64 * t: 64 * (t + 1)] ** 2).sum(1)], 1)
                        for t in range(P)])


def test_gemm_mx8_residual_producer():
    """FC2-style: h += value(a8) value(w8)^T + b in place, with statistics planes and the MX8 copy of h."""
    M, K, N = 777, 3072, 768
    _, a8, as8, A = _acts(M, K, 11, scale=0.3)
    w8, ws8, Wd = _weights(N, K, 12)
    bias = torch.randn(N, device=DEV) * 0.1
    h = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    ref = h.double() + A @ Wd.t() + bias.double()
    ref0 = ref
    P = N // 64
    planes = torch.full((P, M, 2), float("nan"), device=DEV)
    q, s = ops().mx8_empty(M, N, DEV)
    lin = A @ Wd.t() + bias.double()
    vpf().gemm_mx8_res_(a8, as8, w8, ws8, bias, h, planes, q, s)
    _check(h, ref0, lin, A, Wd)
    torch.testing.assert_close(planes.double(), _planes_ref(h, P), rtol=2e-5, atol=2e-3)
    rq, rs = quant(h)
    assert torch.equal(q, rq) and torch.equal(ops().mx8_scale_bytes(s, M), ops().mx8_scale_bytes(rs, M))


@pytest.mark.parametrize("epi", ["res", "patch"])
def test_gemm_bf16_q8_copy(epi):
    """bf16 residual-stream producers (proj, patch embed) with the MX8 copy: equal to quantize(stored rows)."""
    D, K = 768, 768
    if epi == "res":
        M = 600
        a = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
        w = (torch.randn(D, K, device=DEV) * 0.03).to(torch.bfloat16)
        bias = torch.randn(D, device=DEV) * 0.1
        out = torch.randn(M, D, device=DEV).to(torch.bfloat16)
        rows = M
        planes = torch.empty(D // 64, rows, 2, device=DEV)
        q, s = ops().mx8_empty(rows, D, DEV)
        vpf().gemm_q8_(a, w, bias, out, None, 0, E().VPF_EPI_BIAS_RESIDUAL, out, planes, q, s)
        flat = out
        sel = torch.ones(rows, dtype=torch.bool)
    else:
        n, g2 = 3, 196
        a = (torch.randn(n * g2, K, device=DEV) * 0.5).to(torch.bfloat16)
        w = (torch.randn(D, K, device=DEV) * 0.03).to(torch.bfloat16)
        bias = torch.randn(D, device=DEV) * 0.1
        pos = torch.randn(g2 + 1, D, device=DEV) * 0.1
        tok = torch.zeros(n, g2 + 1, D, device=DEV, dtype=torch.bfloat16)
        rows = n * (g2 + 1)
        planes = torch.empty(D // 64, rows, 2, device=DEV)
        q, s = ops().mx8_empty(rows, D, DEV)
        vpf().gemm_q8_(a, w, bias, None, pos, g2, E().VPF_EPI_PATCH, tok, planes, q, s)
        flat = tok.view(rows, D)
        sel = torch.ones(rows, dtype=torch.bool)
        sel[:: g2 + 1] = False          # CLS rows: not written by the GEMM
    rq, rs = quant(flat)
    assert torch.equal(q[sel.to(DEV)], rq[sel.to(DEV)])
    assert torch.equal(ops().mx8_scale_bytes(s, rows)[sel.to(DEV)], ops().mx8_scale_bytes(rs, rows)[sel.to(DEV)])


def test_mx8_argument_contract():
    from vitparticlefiltertracker_amd import _lib
    x = torch.zeros(64, 100, device=DEV, dtype=torch.bfloat16)   # K % 128 != 0
    q = torch.empty(64, 128, device=DEV, dtype=torch.uint8)
    s = torch.empty(1, 64, device=DEV, dtype=torch.int32)
    with pytest.raises(_lib.VPFError):
        _lib.call("vpf_quantize_mx8", x.data_ptr(), 100, 64, 100, 1, q.data_ptr(), 128, s.data_ptr(), 64,
                  _lib.stream_ptr())
    a8, as8 = ops().mx8_empty(64, 128, DEV)
    w8, ws8 = ops().mx8_empty(96, 128, DEV)        # N = 96: scale planes need N % 64 == 0
    with pytest.raises(_lib.VPFError):
        vpf().gemm_mx8(a8, as8, w8, ws8[:, :96].contiguous(), torch.zeros(96, device=DEV), None, None, None,
                       _lib.VPF_EPI_BIAS, torch.empty(64, 96, device=DEV, dtype=torch.bfloat16))
    with pytest.raises(_lib.VPFError):   # EPI_PATCH is not an MX8 epilogue
        w8, ws8 = ops().mx8_empty(128, 128, DEV)
        vpf().gemm_mx8(a8, as8, w8, ws8[:, :128].contiguous(), torch.zeros(128, device=DEV), None, None, None,
                       _lib.VPF_EPI_PATCH, torch.empty(64, 128, device=DEV, dtype=torch.bfloat16))


@pytest.mark.parametrize("B,N,H", [(3, 197, 12), (2, 50, 4)])
def test_attention_mx8_output_matches_quantizer(B, N, H):
    """fp8 path attention: the MX8 output == quantize_mx8 of the bf16 output of the same kernel, bit for bit."""
    D = H * 64
    torch.manual_seed(B * N)
    qkv = (torch.randn(B, N, 3 * D, device=DEV) * 0.7).to(torch.bfloat16)
    out = torch.empty(B, N, D, device=DEV, dtype=torch.bfloat16)
    vpf().attention(qkv, H, N, out)
    q, s = ops().mx8_empty(B * N, D, DEV)
    vpf().attention_q8_(qkv, H, q, s)
    rq, rs = quant(out.view(B * N, D))
    assert torch.equal(q, rq)
    assert torch.equal(ops().mx8_scale_bytes(s, B * N), ops().mx8_scale_bytes(rs, B * N))
