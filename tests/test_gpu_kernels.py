"""GPU (MI355X): every libvpf kernel, called through the product ops / C-ABI, against the oracle (bit-exact
for integer / byte / fixed-function work) or a torch fp32/fp64 reference of the same op (tolerances in
each test). Run: python -m pytest tests -m gpu."""
import numpy as np
import pytest
import torch
import torch.nn.functional as Fn

from oracle import pf

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded():
    from vitparticlefiltertracker_amd import _lib, ops  # noqa: F401
    L = _lib.lib()
    assert b"gfx950" in L.vpf_version()
    assert torch.cuda.is_available()


def vpf():
    return torch.ops.vpf


def bf16_bits(x: np.ndarray) -> np.ndarray:
    """fp32 -> bf16 round-to-nearest-even bit patterns (reference for the bf16 kernels' outputs)."""
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


# ------------------------------------------------------------------ H1 predict
@pytest.mark.parametrize("n,begin", [(1, 0), (1000, 0), (4096, 12288), (65536, 0)])
def test_predict_bit_exact(n, begin):
    rng = np.random.default_rng(n)
    p = np.empty((3, n), np.float32)
    p[0] = rng.uniform(0, 223, n); p[1] = rng.uniform(0, 223, n); p[2] = rng.uniform(0.5, 2.0, n)
    ref = p.copy()
    pf.predict(ref, begin, 1234, 7, (4.0, 4.0, 0.02), 224, 224, (0.5, 2.0))
    d = torch.from_numpy(p).to(DEV)
    vpf().predict_(d, begin, 1234, 7, [4.0, 4.0, 0.02], 224.0, 224.0, [0.5, 2.0])
    got = d.cpu().numpy()
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


# ------------------------------------------------------------------ H2/H3 crop
@pytest.mark.parametrize("box", [(64.0, 48.0), (300.0, 200.0)])
@pytest.mark.parametrize("S,patch,H,W", [(224, 16, 224, 224), (336, 14, 240, 320), (224, 16, 1080, 1920),
                                         (98, 7, 100, 130), (120, 12, 200, 150)])
def test_crop_bit_exact(S, patch, H, W, box):
    """Bit-exact against the oracle. patch 16 takes the LDS-staged kernel (one workgroup per particle, its source
    window in LDS); the (300, 200) box at scale 2 overflows the LDS window and takes its global-tap branch. Patches 14
    and 12 (even, not a multiple of 8: bf16 pair stores) and 7 (odd: element stores) take the per-row kernel."""
    rng = np.random.default_rng(S + H)
    frame = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    n = 5
    p = np.empty((3, n), np.float32)
    p[0] = [W / 2, 0.0, W - 1.0, 13.7, -40.0]
    p[1] = [H / 2, 5.5, H - 1.0, 101.3, -40.0]
    p[2] = [1.0, 0.5, 2.0, 1.37, 1.0]
    kp = (3 * patch * patch + 63) // 64 * 64
    ref = pf.crop_patches(frame, p, box, S, patch, kp, (0.5, 0.4, 0.3), (0.5, 0.25, 0.2))
    from vitparticlefiltertracker_amd.vit import norm_affine
    ab = norm_affine((0.5, 0.4, 0.3), (0.5, 0.25, 0.2))
    a, b = pf.norm_affine((0.5, 0.4, 0.3), (0.5, 0.25, 0.2))
    assert np.array_equal(np.array(ab[:3], np.float32), a) and np.array_equal(np.array(ab[3:], np.float32), b)
    fd, pd = torch.from_numpy(frame).to(DEV), torch.from_numpy(p).to(DEV)
    g = S // patch
    from vitparticlefiltertracker_amd.ops import rgba_workspace
    ws = rgba_workspace((H, W), DEV)
    out32 = torch.empty(n * g * g, kp, device=DEV, dtype=torch.float32)
    vpf().crop_patches(fd, ws, pd, list(box), S, patch, ab, out32)
    assert np.array_equal(out32.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    out16 = torch.empty(n * g * g, kp, device=DEV, dtype=torch.bfloat16)
    vpf().crop_patches(fd, ws, pd, list(box), S, patch, ab, out16)
    assert np.array_equal(out16.cpu().view(torch.int16).numpy().view(np.uint16), bf16_bits(ref))


# ------------------------------------------------------------------ GEMM
def _epi_ref(acc, bias, epi, residual=None):
    y = acc + bias
    if epi == 1:
        y = Fn.gelu(y)
    if epi == 2:
        y = residual.float() + y.to(torch.bfloat16).float()
    return y


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 192, 192), (1000, 768, 768), (513, 2304, 768),
                                   (777, 768, 3072), (64, 520, 128), (4096 * 197 // 64, 3072, 768)])
@pytest.mark.parametrize("epi", [0, 1, 2])
def test_gemm_bf16(M, N, K, epi):
    torch.manual_seed(M * 7 + N + K + epi)
    A = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device=DEV) * 0.1
    R = (torch.randn(M, N, device=DEV)).to(torch.bfloat16) if epi == 2 else None
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    Rin = R.clone() if R is not None else None
    vpf().gemm(A, W, bias, Rin, None, 0, None, None, epi, out)
    ref = _epi_ref(A.float() @ W.float().t(), bias, epi, R)
    torch.testing.assert_close(out.float(), ref, rtol=1.6e-2, atol=1e-2)
    if epi == 2:   # in-place residual (out aliases the residual), as the encoder uses it
        h = R.clone()
        vpf().gemm(A, W, bias, h, None, 0, None, None, epi, h)
        assert torch.equal(h, out)


def test_gemm_bf16_asymmetric_identity():
    """A = I with an asymmetric W catches a transposed C write (cdna_hip_programming.md §3)."""
    M = N = K = 256
    A = torch.eye(M, K, device=DEV, dtype=torch.bfloat16)
    W = (torch.arange(N * K, device=DEV, dtype=torch.float32).reshape(N, K) % 97 - 48).to(torch.bfloat16)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    vpf().gemm(A, W, torch.zeros(N, device=DEV), None, None, 0, None, None, 0, out)
    assert torch.equal(out, W.t().contiguous())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_gemm_patch_epilogue(dtype):
    torch.manual_seed(5)
    n, g2, D, K = 3, 196, 192, 768
    M = n * g2
    A = (torch.randn(M, K, device=DEV) * 0.5).to(dtype)
    W = (torch.randn(D, K, device=DEV) * 0.03).to(dtype)
    bias = torch.randn(D, device=DEV) * 0.1
    pos = torch.randn(g2 + 1, D, device=DEV) * 0.1
    out = torch.full((n, g2 + 1, D), 7.0, device=DEV, dtype=dtype)
    vpf().gemm(A, W, bias, None, pos, g2, None, None, 3, out)
    ref = ((A.double() @ W.double().t()) + bias.double()).reshape(n, g2, D) + pos[1:].double()
    tol = dict(rtol=2e-2, atol=2e-2) if dtype == torch.bfloat16 else dict(rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(out[:, 1:].double(), ref, **tol)
    assert torch.all(out[:, 0] == 7.0)       # CLS rows untouched
    cls = torch.randn(D, device=DEV)
    vpf().cls_rows_(out, cls, pos)
    torch.testing.assert_close(out[:, 0].float(), (cls + pos[0]).expand(n, D).to(dtype).float())


@pytest.mark.parametrize("M,N,K", [(128, 128, 32), (300, 192, 192), (1000, 768, 768)])
@pytest.mark.parametrize("epi", [0, 1, 2])
def test_gemm_f32(M, N, K, epi):
    torch.manual_seed(M + N + K + epi)
    A = torch.randn(M, K, device=DEV)
    W = torch.randn(N, K, device=DEV) / K ** 0.5
    bias = torch.randn(N, device=DEV)
    R = torch.randn(M, N, device=DEV) if epi == 2 else None
    out = torch.empty(M, N, device=DEV)
    vpf().gemm(A, W, bias, R, None, 0, None, None, epi, out)
    acc = A.double() @ W.double().t() + bias.double()
    ref = Fn.gelu(acc) if epi == 1 else (acc + R.double() if epi == 2 else acc)
    torch.testing.assert_close(out.double(), ref, rtol=2e-5, atol=2e-5)


def test_gemm_bf16_gelu_accuracy():
    """The bf16 GEMM's GELU epilogue (sigmoid form, gelu_sig2) against the exact-erf GELU: A W^T is made exact
    (W = I, one nonzero term per output) so the only error left is the GELU's and the bf16 output rounding.
    Bar: |gelu_sig2(x) - gelu(x)| <= 2.8e-4 (the minimax bound) plus half a bf16 ulp of the result."""
    M, K = 4096, 128
    x = torch.linspace(-10, 10, M * K, device=DEV).reshape(M, K).to(torch.bfloat16)
    W = torch.eye(K, device=DEV, dtype=torch.bfloat16)
    bias = torch.zeros(K, device=DEV)
    out = torch.empty(M, K, device=DEV, dtype=torch.bfloat16)
    vpf().gemm(x, W, bias, None, None, 0, None, None, 1, out)
    ref = Fn.gelu(x.double())
    half_ulp = ref.abs().clamp_min(2.0 ** -126) * 2.0 ** -8   # bf16: 8 significant bits
    err = (out.double() - ref).abs()
    assert torch.all(err <= 2.8e-4 + half_ulp), float((err - half_ulp).max())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("gelu", [False, True])
def test_gemm_layernorm_fold(dtype, gelu):
    """EPI_LN / EPI_LN_GELU on the raw rows == LayerNorm -> GEMM(+GELU) (SPEC S4 folded form)."""
    torch.manual_seed(11 + gelu)
    M, D, N = 777, 768, 2304
    h = (torch.randn(M, D, device=DEV) * 1.3 + 0.4).to(dtype)
    g = 1 + 0.2 * torch.randn(D, device=DEV)
    be = 0.1 * torch.randn(D, device=DEV)
    W = torch.randn(N, D, device=DEV) / D ** 0.5
    b = 0.1 * torch.randn(N, device=DEV)
    Wg = (W * g).to(dtype)
    colsum = Wg.float().sum(1)
    bias = b + W @ be
    st = torch.empty(M, 2, device=DEV)
    vpf().row_stats(h, 1e-6, st)
    ref_st = torch.stack([h.double().mean(1), 1 / torch.sqrt(h.double().var(1, unbiased=False) + 1e-6)], 1)
    torch.testing.assert_close(st.double(), ref_st, rtol=1e-5, atol=1e-5)
    out = torch.empty(M, N, device=DEV, dtype=dtype)
    vpf().gemm(h, Wg, bias, None, None, 0, st, colsum, 5 if gelu else 4, out)
    ref = Fn.layer_norm(h.double(), (D,), g.double(), be.double(), 1e-6) @ W.double().t() + b.double()
    if gelu:
        ref = Fn.gelu(ref)
    tol = dict(rtol=2e-2, atol=3e-2) if dtype == torch.bfloat16 else dict(rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(out.double(), ref, **tol)


def _planes_ref(y: torch.Tensor, P: int) -> torch.Tensor:
    """fp64 {sum, sumsq} per 64-column block of the rows of y (the vpf_gemm_bf16 stats_out layout)."""
    yd = y.double()
    out = []
    for t in range(P):
        b = yd[:, 64 * t: 64 * (t + 1)]
        out.append(torch.stack([b.sum(1), (b * b).sum(1)], 1))
    return torch.stack(out)


@pytest.mark.parametrize("M,D", [(777, 768), (300, 192), (513, 960), (512, 1024), (777, 1024)])
def test_gemm_stats_planes(M, D):
    """Residual-stream statistics planes (bf16 LN fold without a row_stats pass): the EPI_BIAS_RESIDUAL producer
    writes {sum, sumsq} of its stored bf16 rows per 256-column block; an EPI_LN consumer reading those planes
    (stats_parts = P, ln_eps) equals LayerNorm -> GEMM on the same rows. D = 1024 (16 planes, ViT-L) takes the
    consumer's wide path (planes land in a free operand slot at the last K-step)."""
    torch.manual_seed(M + D)
    P = (D + 63) // 64
    x = (torch.randn(M, D, device=DEV) * 0.7).to(torch.bfloat16)
    W = (torch.randn(D, D, device=DEV) / D ** 0.5).to(torch.bfloat16)
    bias = torch.randn(D, device=DEV) * 0.1
    h = (torch.randn(M, D, device=DEV) + 0.3).to(torch.bfloat16)
    planes = torch.full((P, M, 2), float("nan"), device=DEV)
    vpf().gemm_stats_(x, W, bias, h, None, 0, 2, h, planes)
    torch.testing.assert_close(planes.double(), _planes_ref(h, P), rtol=2e-5, atol=2e-3)
    # consumer: LN folded GEMM reading the planes
    N = 2 * D
    g = 1 + 0.2 * torch.randn(D, device=DEV)
    be = 0.1 * torch.randn(D, device=DEV)
    W2 = torch.randn(N, D, device=DEV) / D ** 0.5
    b2 = 0.1 * torch.randn(N, device=DEV)
    Wg = (W2 * g).to(torch.bfloat16)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    vpf().gemm(h, Wg, b2 + W2 @ be, None, None, 0, planes, Wg.float().sum(1), 4, out, P, 1e-6)
    ref = Fn.layer_norm(h.double(), (D,), g.double(), be.double(), 1e-6) @ W2.double().t() + b2.double()
    torch.testing.assert_close(out.double(), ref, rtol=2e-2, atol=3e-2)


@pytest.mark.parametrize("M,D,N,epi", [(4099, 1024, 3072, 4), (2500, 1024, 4096, 5), (777, 768, 2304, 4),
                                         (1, 192, 576, 4), (257, 192, 768, 5)])
def test_stats_combine_equals_in_kernel_combine(M, D, N, epi):
    """vpf_stats_combine (round 5): the producer's statistics planes combined into {mean, rstd} by a separate pass, then
    the LN-folded GEMM with stats_parts = 0 (ViT-L's 16 planes then run the ping-pong kernel), gives the same bits as the
    GEMM combining the planes itself (16 planes: kernel 1's wide form; 12: the ping-pong kernel's)."""
    torch.manual_seed(M + D)
    P = D // 64
    h = (torch.randn(M, D, device=DEV) + 0.3).to(torch.bfloat16)
    planes = _planes_ref(h, P).float().contiguous()
    W = (torch.randn(N, D, device=DEV) / D ** 0.5).to(torch.bfloat16)
    bias = 0.1 * torch.randn(N, device=DEV)
    colsum = W.float().sum(1).contiguous()
    ref = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    vpf().gemm(h, W, bias, None, None, 0, planes, colsum, epi, ref, P, 1e-6)
    st = torch.empty(M, 2, device=DEV)
    vpf().stats_combine_(planes, D, 1e-6, st)
    got = torch.empty_like(ref)
    vpf().gemm(h, W, bias, None, None, 0, st, colsum, epi, got)
    assert torch.equal(got, ref)
    mean, var = h.double().mean(1), h.double().var(1, unbiased=False)
    torch.testing.assert_close(st.double(), torch.stack([mean, 1 / torch.sqrt(var + 1e-6)], 1), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("M,N,K,P", [(777, 768, 768, 12), (1000, 2304, 3072, 12), (806912 // 8, 3072, 768, 12),
                                     (3001, 2304, 64, 12), (4099, 1024, 192, 16)])
def test_gemm_kernel_variants_bit_identical(M, N, K, P):
    """The product library's two bf16 GEMM kernels (vpf_gemm_tune 1 = the deep-ring k_gemm_bf16, 5 = the ping-pong
    k_gemm_pp, which QKV runs by default) accumulate each output over the same K order, so they give the same bits for
    every epilogue: bias, bias+GELU, residual with statistics planes, patch rows, LN fold, LN fold + GELU (12 planes,
    or ViT-L's 16: kernel 5 then falls back to kernel 1's wide form). M is not a multiple of the 256-row tile (edge
    tiles); nk = 1 and 3 are the shortest K loops. Kernel 0 = the per-shape defaults the product runs."""
    from vitparticlefiltertracker_amd import _lib
    L = _lib.lib()
    torch.manual_seed(M + N + K)
    A = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device=DEV) * 0.1
    R = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    colsum = W.float().sum(1).contiguous()
    planes_in = torch.stack([torch.randn(P, M, device=DEV) * 3.0, torch.rand(P, M, device=DEV) * 60 + 40], 2)
    planes_in = planes_in.contiguous()
    g2 = 196 if M % 196 == 0 else 1
    pos = torch.randn(g2 + 1, N, device=DEV)

    def run(epi):
        if epi == 3:
            out = torch.zeros(M // g2 * (g2 + 1), N, device=DEV, dtype=torch.bfloat16)
            vpf().gemm(A, W, bias, None, pos, g2, None, None, 3, out)
            return out, None
        out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        if epi == 2:
            out.copy_(R)
            st = torch.zeros((N + 63) // 64, M, 2, device=DEV)
            vpf().gemm_stats_(A, W, bias, out, None, 0, 2, out, st)
            return out, st
        if epi in (4, 5):
            vpf().gemm(A, W, bias, None, None, 0, planes_in, colsum, epi, out, P, 1e-6)
        else:
            vpf().gemm(A, W, bias, None, None, 0, None, None, epi, out)
        return out, None

    try:
        for epi in (0, 1, 2, 3, 4, 5):
            assert L.vpf_gemm_tune(1, -1) == 0
            ref, ref_st = run(epi)
            for k, g in ((0, -1), (5, -1), (1, 0), (5, 8)):
                assert L.vpf_gemm_tune(k, g) == 0
                got, st = run(epi)
                torch.cuda.synchronize()
                bad = (got.view(torch.int16) != ref.view(torch.int16)).sum().item()
                assert bad == 0, (k, g, epi, bad)
                if ref_st is not None:
                    assert torch.equal(st, ref_st), (k, epi)
    finally:
        L.vpf_gemm_tune(0, -1)                # the per-shape defaults


@pytest.mark.parametrize("epi", [1, 4, 5])
@pytest.mark.parametrize("kern", [1, 5])
def test_gemm_single_k_tile_epilogues_vs_fp64(epi, kern):
    """K = 64 (one K-tile, nk = 1): the epilogue operands (bias, colsum, statistics planes) are DMA'd by some waves and
    read by all, so they must land before the loop's only barrier (the deep-ring kernel issued them after
    it, and its direct-store GELU epilogue could read stale bias). Bias + GELU, LN fold and LN fold + GELU on both
    product kernels against float64, over 4096 tiles and three repeats with different bias values each time (a stale
    read shows as a wrong column block)."""
    from vitparticlefiltertracker_amd import _lib
    L = _lib.lib()
    M, N, K, P = 256 * 128, 8192, 64, 1
    torch.manual_seed(epi * 10 + kern)
    A = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    colsum = W.float().sum(1).contiguous()
    st = torch.stack([torch.randn(M, device=DEV) * 0.1, torch.rand(M, device=DEV) + 0.5], 1).contiguous()
    try:
        assert L.vpf_gemm_tune(kern, -1) == 0
        for rep in range(3):
            bias = (torch.randn(N, device=DEV) * (rep + 1)).contiguous()
            out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            if epi == 1:
                vpf().gemm(A, W, bias, None, None, 0, None, None, 1, out)
                ref = Fn.gelu(A.double() @ W.double().t() + bias.double())
            else:
                vpf().gemm(A, W, bias, None, None, 0, st, colsum, epi, out)
                mean, rstd = st[:, 0].double(), st[:, 1].double()
                ref = rstd[:, None] * (A.double() @ W.double().t()) - (rstd * mean)[:, None] * colsum.double() \
                    + bias.double()
                if epi == 5:
                    ref = Fn.gelu(ref)
            torch.testing.assert_close(out.double(), ref, rtol=1.6e-2, atol=2e-2)
    finally:
        L.vpf_gemm_tune(0, -1)


def test_patch_and_cls_stats_planes():
    """EPI_PATCH + vpf_cls_rows_bf16 together fill the planes of every token row (patch rows by the GEMM, CLS
    rows by cls_rows), matching the stored bf16 token rows."""
    torch.manual_seed(5)
    n, g2, D, K = 5, 196, 768, 768
    P = 12
    A = (torch.randn(n * g2, K, device=DEV) * 0.5).to(torch.bfloat16)
    W = (torch.randn(D, K, device=DEV) * 0.03).to(torch.bfloat16)
    bias = torch.randn(D, device=DEV) * 0.1
    pos = torch.randn(g2 + 1, D, device=DEV) * 0.1
    cls = torch.randn(D, device=DEV)
    tok = torch.empty(n, g2 + 1, D, device=DEV, dtype=torch.bfloat16)
    planes = torch.full((P, n * (g2 + 1), 2), float("nan"), device=DEV)
    vpf().gemm_stats_(A, W, bias, None, pos, g2, 3, tok, planes)
    vpf().cls_rows_stats_(tok, cls, pos, planes)
    ref = _planes_ref(tok.view(-1, D), P)
    patch_rows = torch.ones(n * (g2 + 1), dtype=torch.bool)
    patch_rows[:: g2 + 1] = False
    torch.testing.assert_close(planes[:, patch_rows].double(), ref[:, patch_rows], rtol=2e-5, atol=2e-3)
    # CLS rows: the whole row's {sum, sumsq} in plane 0, zeros elsewhere (the consumer sums the planes)
    torch.testing.assert_close(planes[0, ~patch_rows].double(), ref[:, ~patch_rows].sum(0), rtol=2e-5, atol=2e-3)
    assert torch.all(planes[1:, ~patch_rows] == 0)


@pytest.mark.parametrize("case", ["offset", "outliers"])
def test_gemm_stats_planes_cancellation(case):
    """The planes consumer takes var = sum(sumsq)/D - mean^2 in one pass (fp32); the row_stats path and the
    oracle take it in two passes. Residual rows with a large common offset (|mean| = 8 std) or a few
    large-magnitude channels (ViT's outlier dimensions, 40-60x the rest) must give the same LN-folded GEMM
    output as the two-pass path within bf16 output rounding (parity there was unpinned)."""
    torch.manual_seed(21)
    M, D = 777, 768
    P = D // 64
    hf = torch.randn(M, D, device=DEV)
    if case == "offset":
        hf = hf + 8.0
    else:
        idx = torch.tensor([3, 200, 411, 767], device=DEV)
        hf[:, idx] = hf[:, idx] * 4 + torch.tensor([60.0, -45.0, 52.0, -40.0], device=DEV)
    x = (torch.randn(M, D, device=DEV) * 0.7).to(torch.bfloat16)
    W = (torch.randn(D, D, device=DEV) / D ** 0.5).to(torch.bfloat16)
    bias = torch.randn(D, device=DEV) * 0.1
    h = hf.to(torch.bfloat16)
    planes = torch.empty((P, M, 2), device=DEV)
    # producer writes h in place as h + x W^T + bias; the planes describe the stored rows
    vpf().gemm_stats_(x, W, bias, h, None, 0, 2, h, planes)
    N = 2 * D
    g = 1 + 0.2 * torch.randn(D, device=DEV)
    be = 0.1 * torch.randn(D, device=DEV)
    W2 = torch.randn(N, D, device=DEV) / D ** 0.5
    b2 = 0.1 * torch.randn(N, device=DEV)
    Wg = (W2 * g).to(torch.bfloat16)
    cs = Wg.float().sum(1)
    out_planes = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    vpf().gemm(h, Wg, b2 + W2 @ be, None, None, 0, planes, cs, 4, out_planes, P, 1e-6)
    st = torch.empty(M, 2, device=DEV)
    vpf().row_stats(h, 1e-6, st)
    out_twopass = torch.empty_like(out_planes)
    vpf().gemm(h, Wg, b2 + W2 @ be, None, None, 0, st, cs, 4, out_twopass)
    ref = Fn.layer_norm(h.double(), (D,), g.double(), be.double(), 1e-6) @ W2.double().t() + b2.double()
    torch.testing.assert_close(out_planes.double(), ref, rtol=2e-2, atol=3e-2)
    # one-pass vs two-pass statistics: the same output up to a few bf16 ulps (relative Frobenius error)
    rel = ((out_planes.double() - out_twopass.double()).norm() / out_twopass.double().norm()).item()
    rel_ref = ((out_twopass.double() - ref).norm() / ref.norm()).item()
    assert rel < 4e-3 and rel < 2 * rel_ref + 1e-4, (rel, rel_ref)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_gemm_strided_rows(dtype):
    """a / out / residual as row-strided views (the last layer's CLS rows of the token tensor)."""
    torch.manual_seed(12)
    n, Ntok, D, F = 300, 197, 768, 3072
    tok = torch.randn(n, Ntok, D, device=DEV).to(dtype)
    hid = torch.empty(n, F, device=DEV, dtype=dtype)
    W1 = (torch.randn(F, D, device=DEV) / D ** 0.5).to(dtype)
    b1 = torch.randn(F, device=DEV) * 0.1
    cls = tok.view(n, Ntok * D)[:, :D]
    vpf().gemm(cls, W1, b1, None, None, 0, None, None, 1, hid)
    ref = Fn.gelu(tok[:, 0].double() @ W1.double().t() + b1.double())
    tol = dict(rtol=2e-2, atol=2e-2) if dtype == torch.bfloat16 else dict(rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(hid.double(), ref, **tol)
    W2 = (torch.randn(D, F, device=DEV) / F ** 0.5).to(dtype)
    b2 = torch.randn(D, device=DEV) * 0.1
    before = tok.clone()
    vpf().gemm(hid, W2, b2, cls, None, 0, None, None, 2, cls)
    ref2 = before[:, 0].double() + (hid.double() @ W2.double().t() + b2.double())
    torch.testing.assert_close(tok[:, 0].double(), ref2, **tol)
    assert torch.equal(tok[:, 1:], before[:, 1:])          # non-CLS rows untouched


# ------------------------------------------------------------------ LayerNorm
@pytest.mark.parametrize("rows,D", [(1, 192), (1000, 768), (333, 1024), (64, 4)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_layernorm(rows, D, dtype):
    torch.manual_seed(rows + D)
    x = (torch.randn(rows, D, device=DEV) * 2 + 0.5).to(dtype)
    g = 1 + 0.1 * torch.randn(D, device=DEV)
    b = 0.1 * torch.randn(D, device=DEV)
    y = torch.empty_like(x)
    vpf().layernorm(x, g, b, 1e-6, y)
    ref = Fn.layer_norm(x.double(), (D,), g.double(), b.double(), 1e-6)
    tol = dict(rtol=1e-2, atol=2e-2) if dtype == torch.bfloat16 else dict(rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(y.double(), ref, **tol)
    # row-strided input / output views
    big = torch.zeros(rows, 3 * D, device=DEV, dtype=dtype)
    big[:, D:2 * D] = x
    ys = torch.zeros(rows, 2 * D, device=DEV, dtype=dtype)
    vpf().layernorm(big[:, D:2 * D], g, b, 1e-6, ys[:, :D])
    assert torch.equal(ys[:, :D], y) and torch.all(ys[:, D:] == 0)
    if D % 8 == 0:
        st = torch.empty(rows, 2, device=DEV)
        vpf().row_stats(big[:, D:2 * D], 1e-6, st)
        ref_st = torch.stack([x.double().mean(1), 1 / torch.sqrt(x.double().var(1, unbiased=False) + 1e-6)], 1)
        torch.testing.assert_close(st.double(), ref_st, rtol=1e-5, atol=1e-5)


# ------------------------------------------------------------------ attention
@pytest.mark.parametrize("B,N,H", [(3, 197, 12), (2, 577, 16), (5, 1, 3), (4, 64, 2), (2, 100, 1)])
def test_attention_bf16(B, N, H):
    torch.manual_seed(B * N + H)
    D = 64 * H
    qkv = (torch.randn(B, N, 3 * D, device=DEV) * 1.5).to(torch.bfloat16)
    out = torch.empty(B, N, D, device=DEV, dtype=torch.bfloat16)
    vpf().attention(qkv, H, N, out)
    q, k, v = qkv.float().reshape(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    ref = torch.softmax((q @ k.transpose(-1, -2)) * 0.125, -1) @ v
    ref = ref.transpose(1, 2).reshape(B, N, D)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,N,H", [(4, 197, 3), (3, 577, 16), (2, 40, 2)])
def test_attention_q_rows(dtype, B, N, H):
    """q_rows = 1 (last block: CLS query only) and q_rows = 2 (first strip, partial). bf16 q_rows = 1 runs the
    dedicated fp32-softmax CLS kernel: checked against an fp64 reference; the rows it must not touch stay
    untouched. q_rows = 2, q_rows = N - 1 (the last query row left out: at N = 577 the 16-query strip's one row) and
    fp32 are the same code as the full call: bit-equal."""
    torch.manual_seed(3)
    D = 64 * H
    qkv = torch.randn(B, N, 3 * D, device=DEV).to(dtype)
    full = torch.empty(B, N, D, device=DEV, dtype=dtype)
    vpf().attention(qkv, H, N, full)
    q, k, v = qkv.double().reshape(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    ref = (torch.softmax((q @ k.transpose(-1, -2)) * 0.125, -1) @ v).transpose(1, 2).reshape(B, N, D)
    part = torch.full((B, N, D), 5.0, device=DEV, dtype=dtype)
    vpf().attention(qkv, H, 1, part)
    if dtype == torch.bfloat16:
        torch.testing.assert_close(part[:, 0].double(), ref[:, 0], rtol=1e-2, atol=1e-2)
    else:
        assert torch.equal(part[:, 0], full[:, 0])
    assert torch.all(part[:, 1:] == 5.0)
    part2 = torch.full((B, N, D), 5.0, device=DEV, dtype=dtype)
    vpf().attention(qkv, H, 2, part2)
    assert torch.equal(part2[:, :2], full[:, :2])
    assert torch.all(part2[:, 2:] == 5.0)
    part3 = torch.full((B, N, D), 5.0, device=DEV, dtype=dtype)
    vpf().attention(qkv, H, N - 1, part3)
    assert torch.equal(part3[:, :N - 1], full[:, :N - 1])
    assert torch.all(part3[:, N - 1:] == 5.0)


@pytest.mark.parametrize("B,N,H", [(3, 197, 12), (5, 197, 6), (2, 256, 12), (4, 1, 6), (64, 50, 12), (2, 577, 16),
                                   (3, 640, 16)])
def test_cls_attn_fold(B, N, H):
    """The last block's CLS attention with K / V never formed (vpf_cls_attn_fold_bf16) against an fp64
    restatement: LNraw from the statistics planes, s_hj = (LNraw_j . G_h + q_h . bk_h) / 8, U_h = sum_j p_hj
    LNraw_j. Then the whole identity: W'_v,h U_h + b'_v equals the explicit softmax(q k^T / 8) v with
    k, v = LN(h) W'^T + b' (tolerance: bf16 rounding of LNraw in the dots and of the output)."""
    torch.manual_seed(B * N + H)
    D = 64 * H
    h = (torch.randn(B, N, D, device=DEV) * 1.3 + 0.2).to(torch.bfloat16)
    planes = _planes_ref(h.view(B * N, D), H).float().contiguous()
    Wk = torch.randn(D, D, device=DEV) / D ** 0.5
    Wv = torch.randn(D, D, device=DEV) / D ** 0.5
    bk = 0.3 * torch.randn(D, device=DEV)
    bv = 0.3 * torch.randn(D, device=DEV)
    qall = (torch.randn(B, 2, D, device=DEV) * 3.0).to(torch.bfloat16)   # scores of std ~3: a peaked softmax
    q = qall[:, 0]                                        # row-strided view (row stride 2D), as in vit.py
    qd = q.double().reshape(B, H, 64)
    G = torch.einsum("bhd,hdi->bhi", qd, Wk.double().view(H, 64, D)).to(torch.bfloat16).contiguous()   # [B][H][D]
    out = torch.full((B, H * D), float("nan"), device=DEV, dtype=torch.bfloat16)
    vpf().cls_attn_fold_(h, planes, 1e-6, G.view(B, H * D), q, bk, H, out)
    hd_ = h.double()
    mean = hd_.mean(-1, keepdim=True)
    var = (hd_ * hd_).mean(-1, keepdim=True) - mean * mean
    ln = (hd_ - mean) / torch.sqrt(var + 1e-6)                                            # [B][N][D]
    c0 = (qd * bk.double().view(H, 64)).sum(-1)                                           # [B][H]
    s = (torch.einsum("bnd,bhd->bhn", ln, G.double()) + c0[..., None]) * 0.125
    p = torch.softmax(s, -1)
    U = torch.einsum("bhn,bnd->bhd", p, ln)
    torch.testing.assert_close(out.double().view(B, H, D), U, rtol=2e-2, atol=1e-2 * U.abs().max().item())
    # the algebra: W'_v,h U_h + b'_v == softmax(q k^T / 8) v on the explicit K, V
    k = (ln @ Wk.double().t() + bk.double()).view(B, N, H, 64)
    v = (ln @ Wv.double().t() + bv.double()).view(B, N, H, 64)
    att = torch.softmax(torch.einsum("bhd,bnhd->bhn", qd, k) * 0.125, -1)
    o_ref = torch.einsum("bhn,bnhd->bhd", att, v)
    o = torch.einsum("bhi,hdi->bhd", out.double().view(B, H, D), Wv.double().view(H, 64, D)) + bv.double().view(H, 64)
    torch.testing.assert_close(o, o_ref, rtol=3e-2, atol=2e-2 * o_ref.abs().max().item())


@pytest.mark.parametrize("n,H", [(5, 12), (1, 6), (33, 16)])
def test_head_gather(n, H):
    """vpf_head_gather_bf16: out[p][h hd + d] = Y[p H + h][h hd + d], into row-strided output; bit-exact."""
    D = 64 * H
    Y = torch.randn(n * H, D, device=DEV).to(torch.bfloat16)
    big = torch.full((n, 3 * D), 9.0, device=DEV, dtype=torch.bfloat16)
    out = big[:, D:2 * D]
    vpf().head_gather_(Y, H, out)
    ref = torch.stack([Y.view(n, H, D)[:, h, 64 * h:64 * h + 64] for h in range(H)], 1).reshape(n, D)
    assert torch.equal(out, ref)
    assert torch.all(big[:, :D] == 9.0) and torch.all(big[:, 2 * D:] == 9.0)


def test_cls_attn_fold_argument_contract():
    H, D, B, N = 12, 768, 2, 197
    h = torch.zeros(B, N, D, device=DEV, dtype=torch.bfloat16)
    planes = torch.zeros(H, B * N, 2, device=DEV)
    G = torch.zeros(B, H * D, device=DEV, dtype=torch.bfloat16)
    q = torch.zeros(B, D, device=DEV, dtype=torch.bfloat16)
    bk = torch.zeros(D, device=DEV)
    out = torch.empty(B, H * D, device=DEV, dtype=torch.bfloat16)
    from vitparticlefiltertracker_amd._lib import VPFError
    with pytest.raises((ValueError, VPFError)):
        vpf().cls_attn_fold_(h, planes[:, :B * N - 1], 1e-6, G, q, bk, H, out)       # planes too short
    h8 = torch.zeros(B, N, 512, device=DEV, dtype=torch.bfloat16)
    with pytest.raises((ValueError, VPFError)):
        vpf().cls_attn_fold_(h8, torch.zeros(8, B * N, 2, device=DEV), 1e-6, torch.zeros(B, 8 * 512, device=DEV,
                             dtype=torch.bfloat16), torch.zeros(B, 512, device=DEV, dtype=torch.bfloat16),
                             torch.zeros(512, device=DEV), 8, torch.empty(B, 8 * 512, device=DEV,
                                                                          dtype=torch.bfloat16))   # H = 8
    h700 = torch.zeros(1, 700, D, device=DEV, dtype=torch.bfloat16)
    with pytest.raises((ValueError, VPFError)):
        vpf().cls_attn_fold_(h700, torch.zeros(H, 700, 2, device=DEV), 1e-6, G[:1], q[:1], bk, H, out[:1])  # N > 640


def _attn_ref64(qkv, H):
    B, N = qkv.shape[0], qkv.shape[1]
    q, k, v = qkv.double().reshape(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    return (torch.softmax((q @ k.transpose(-1, -2)) * 0.125, -1) @ v).transpose(1, 2).reshape(B, N, H * 64)


@pytest.mark.parametrize("B,N,H", [(100, 197, 12), (90, 256, 12), (96, 280, 12), (80, 111, 12), (70, 33, 6),
                                   (4096, 197, 12), (64, 577, 16), (40, 400, 8), (30, 640, 16), (50, 300, 12),
                                   (60, 257, 12), (40, 520, 16), (40, 545, 8)])
def test_attention_bf16_large(B, N, H):
    """B*H >= 4 x CUs; (4096, 197, 12) is the configs[1] launch. N <= 256 runs the key-pipelined kernel (with the
    16-query tail strip when the last strip holds <= 16 real queries: N = 197 / 111 / 33). N > 256 runs the key-streamed
    kernel: 4-wave workgroups of 4 x 32-query strips, four per CU (round 6), K / V through a ring of 4 chunk slots (2
    groups of 2 chunks), one strip kind per wave. N = 577 (configs[3], 64 x 16 units): 5 blocks, the last with 2
    strips and the 16-query strip of query 576 on a wave of its own; N = 400 / 520: 12 / 16 full strips, so the host
    adds a block whose wave 0 runs the 16-query strip (16 / 8 tail queries) alone; N = 300 / 545: the 16-query strip on
    a free wave of the last block (12 / 1 tail queries); N = 257: 8 full strips, the added block's 16-query strip holds
    one query, and the last chunk one real key (the 8-key tail step); N = 280: a partial 32-query strip; N = 640: 5 full blocks. Against an fp64 reference
    on at most 512 particles:
    every element within bf16 output rounding plus the bf16 probabilities' error, and no non-finite value anywhere
    (the round-2 stale-register NaN). q_rows = 1 (the CLS kernel) likewise."""
    torch.manual_seed(N + H)
    D = 64 * H
    qkv = (torch.randn(B, N, 3 * D, device=DEV) * 1.5).to(torch.bfloat16)
    out = torch.empty(B, N, D, device=DEV, dtype=torch.bfloat16)
    vpf().attention(qkv, H, N, out)
    assert torch.isfinite(out.float()).all()
    sub = slice(0, min(B, 512))
    ref = _attn_ref64(qkv[sub], H)
    torch.testing.assert_close(out[sub].double(), ref, rtol=2e-2, atol=2e-2)
    # a second launch gives the same bits (no dependence on timing / co-resident workgroups)
    again = torch.empty_like(out)
    vpf().attention(qkv, H, N, again)
    assert torch.equal(out, again)
    part = torch.full((B, N, D), 5.0, device=DEV, dtype=torch.bfloat16)
    vpf().attention(qkv, H, 1, part)
    torch.testing.assert_close(part[sub, 0].double(), ref[:, 0], rtol=1e-2, atol=1e-2)
    assert torch.all(part[:, 1:] == 5.0)


def test_attention_bf16_rescale_branch():
    """The lazy online-softmax rescale only runs when a query's max grows by > 2^8 (exp2 domain) within a
    key tile: force it (a key row aligned with a query, late in the sequence) and also plant spikes below the
    threshold, then check against a full fp64 reference (cdna_hip_programming.md §5.4 rule 26), on the key-pipelined
    kernel (N = 197) and the key-streamed one (N = 300, 577). Since round 5 a step exponentiates against the running
    max first and redoes the step only when a lane's probabilities sum past 2^8: the spike rows force that redo."""
    torch.manual_seed(26)
    for B, N, H in ((100, 197, 12), (40, 300, 12), (40, 577, 16)):
        D = 64 * H
        qkv = (torch.randn(B, N, 3 * D, device=DEV) * 0.5).to(torch.bfloat16)
        for b in range(0, B, 7):
            h = b % H
            q = qkv[b, 5, h * 64:(h + 1) * 64].float()
            qkv[b, 150, D + h * 64:D + (h + 1) * 64] = (q * 12.0).to(torch.bfloat16)       # far past the threshold
            qkv[b, 40, D + h * 64:D + (h + 1) * 64] = (q * 1.5).to(torch.bfloat16)         # moderate, below it
            qkv[b, N - 1, D + h * 64:D + (h + 1) * 64] = (q * 20.0).to(torch.bfloat16)     # in the masked tail tile
        out = torch.empty(B, N, D, device=DEV, dtype=torch.bfloat16)
        vpf().attention(qkv, H, N, out)
        torch.testing.assert_close(out.double(), _attn_ref64(qkv, H), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("B,N,H", [(2, 197, 3), (1, 50, 2), (1, 577, 2)])
def test_attention_f32(B, N, H):
    torch.manual_seed(N)
    D = 64 * H
    qkv = torch.randn(B, N, 3 * D, device=DEV)
    out = torch.empty(B, N, D, device=DEV)
    vpf().attention(qkv, H, N, out)
    q, k, v = qkv.double().reshape(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    ref = (torch.softmax((q @ k.transpose(-1, -2)) * 0.125, -1) @ v).transpose(1, 2).reshape(B, N, D)
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-5)


# ------------------------------------------------------------------ H9/H10 weights
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_cls_weight(dtype):
    torch.manual_seed(9)
    n, N, D = 257, 5, 768
    tok = torch.randn(n, N, D, device=DEV).to(dtype)
    g = 1 + 0.1 * torch.randn(D, device=DEV)
    b = 0.1 * torch.randn(D, device=DEV)
    t = torch.randn(D, device=DEV)
    t = t / t.norm()
    Q = torch.empty(n, device=DEV, dtype=torch.int64)
    feat = torch.empty(n, D, device=DEV)
    sim = torch.empty(n, device=DEV)
    vpf().cls_weight(tok, g, b, 1e-6, t, 20.0, 40, Q, feat, sim)
    f_ref = Fn.layer_norm(tok[:, 0].double(), (D,), g.double(), b.double(), 1e-6)
    torch.testing.assert_close(feat.double(), f_ref, rtol=1e-5, atol=1e-5)
    s_ref = (f_ref @ t.double()) / f_ref.norm(dim=1)
    torch.testing.assert_close(sim.double(), s_ref, rtol=0, atol=2e-6)
    # Q is the exact SPEC S5 function of the kernel's own sim (fixed expf, floor at 2^40)
    q_ref = pf.weights_to_Q(sim.cpu().numpy(), 20.0, 40)
    assert np.array_equal(Q.cpu().numpy(), q_ref)
    # explicit-feature path (ParticleFilter.update)
    Q2 = torch.empty_like(Q)
    vpf().cosine_weight(feat, t, 20.0, 40, Q2, None)
    assert np.array_equal(Q2.cpu().numpy(), q_ref)


def test_cosine_weight_edge_rows():
    """SPEC S5 guards: a feature row parallel to the template (fp32 sim may round above 1) still gets
    Q <= 2^K; rows with NaN / inf get Q = 0; a zero row gets sim 0; an antiparallel row gets exp(-2 lam).
    Negative or non-finite lambda is rejected by the C-ABI."""
    torch.manual_seed(4)
    D, K = 768, 40
    t = torch.randn(D, device=DEV)
    t = t / t.norm()
    rows = [t * 3.7, t * 1e-3, t, -t, torch.zeros(D, device=DEV), torch.randn(D, device=DEV)]
    bad = torch.randn(D, device=DEV); bad[5] = float("nan"); rows.append(bad)
    bad = torch.randn(D, device=DEV); bad[9] = float("inf"); rows.append(bad)
    for k in range(24):                            # near-parallel rows: rounding can push sim past 1
        rows.append(t * (0.5 + k) + 1e-7 * torch.randn(D, device=DEV))
    feat = torch.stack(rows).contiguous()
    Q = torch.empty(feat.shape[0], device=DEV, dtype=torch.int64)
    sim = torch.empty(feat.shape[0], device=DEV)
    vpf().cosine_weight(feat, t, 20.0, K, Q, sim)
    q = Q.cpu().numpy()
    assert q.max() <= 2 ** K and q.min() >= 0
    assert q[6] == 0 and q[7] == 0                 # non-finite rows
    s_host = sim.cpu().numpy()
    assert np.isnan(s_host[6]) and np.isnan(s_host[7]) and s_host[4] == 0
    assert np.array_equal(q, pf.weights_to_Q(sim.cpu().numpy(), 20.0, K))
    assert q[0] == 2 ** K or q[0] >= 2 ** K - 2 ** 18
    with pytest.raises(Exception):
        vpf().cosine_weight(feat, t, -1.0, K, Q, None)
    with pytest.raises(Exception):
        vpf().cosine_weight(feat, t, float("inf"), K, Q, None)


# ------------------------------------------------------------------ H11/H12
def test_shard_stats():
    rng = np.random.default_rng(3)
    n = 5000
    Q = rng.integers(0, 1 << 40, n, dtype=np.int64)
    p = rng.uniform(0, 224, (3, n)).astype(np.float32)
    T, sums = pf.shard_stats(Q, p)
    To = torch.empty(1, device=DEV, dtype=torch.int64)
    So = torch.empty(3, device=DEV, dtype=torch.float64)
    vpf().shard_stats(torch.from_numpy(Q).to(DEV), torch.from_numpy(p).to(DEV), To, So)
    assert int(To.item()) == T
    np.testing.assert_allclose(So.cpu().numpy(), sums, rtol=1e-13)


@pytest.mark.parametrize("P", [1, 2, 7, 4096, 65536])
@pytest.mark.parametrize("mode", ["dense", "sparse", "zero", "onehot"])
def test_resample_bit_exact(P, mode):
    rng = np.random.default_rng(P)
    Q = rng.integers(0, 1 << 40, P, dtype=np.int64)
    if mode == "sparse":
        Q[rng.random(P) < 0.9] = 0
    if mode == "zero":
        Q[:] = 0
    if mode == "onehot":
        Q[:] = 0
        Q[P // 3] = 12345
    p = rng.uniform(0, 224, (3, P)).astype(np.float32)
    U = int(rng.integers(0, 2 ** 32))
    ref = pf.resample(Q, U)
    from vitparticlefiltertracker_amd.particle_filter import plan_resample
    uniform, T, offs, ranges = plan_resample([(int(Q.sum()), 0, 0, 0)], P, P, U)
    anc = torch.empty(P, device=DEV, dtype=torch.int32)
    states = torch.empty(3, P, device=DEV)
    cdf = torch.empty(P, device=DEV, dtype=torch.int64)
    pd = torch.from_numpy(p).to(DEV)
    vpf().resample(torch.from_numpy(Q).to(DEV), 0, 0, T, P, U, uniform, 0, P, pd, anc, states, cdf)
    assert np.array_equal(anc.cpu().numpy(), ref)
    assert np.array_equal(states.cpu().numpy(), p[:, ref])


@pytest.mark.parametrize("G", [2, 4, 8])
def test_resample_sharded_equals_global(G):
    """Per-shard kernel calls with the host plan reproduce the global ancestors (bit-exact, any G)."""
    from vitparticlefiltertracker_amd.particle_filter import plan_resample
    rng = np.random.default_rng(G)
    P = 4096
    n = P // G
    Q = rng.integers(0, 1 << 40, P, dtype=np.int64)
    Q[rng.random(P) < 0.7] = 0
    p = rng.uniform(0, 224, (3, P)).astype(np.float32)
    U = int(rng.integers(0, 2 ** 32))
    ref = pf.resample(Q, U)
    stats = [(int(Q[r * n:(r + 1) * n].sum()), 0, 0, 0) for r in range(G)]
    uniform, T, offs, ranges = plan_resample(stats, P, n, U)
    got = []
    for r in range(G):
        a, b = ranges[r]
        if b == a:
            continue
        anc = torch.empty(b - a, device=DEV, dtype=torch.int32)
        st = torch.empty(3, b - a, device=DEV)
        cdf = torch.empty(n, device=DEV, dtype=torch.int64)
        vpf().resample(torch.from_numpy(Q[r * n:(r + 1) * n].copy()).to(DEV), r * n, offs[r], T, P, U, uniform, a, b,
                       torch.from_numpy(p[:, r * n:(r + 1) * n].copy()).to(DEV), anc, st, cdf)
        got.append(anc.cpu().numpy())
    assert np.array_equal(np.concatenate(got), ref)


@pytest.mark.parametrize("G", [1, 2, 8])
@pytest.mark.parametrize("P,mode", [(7, "dense"), (4096, "dense"), (4096, "sparse"), (4096, "zero"),
                                    (4096, "onehot"), (65536, "sparse")])
def test_estimate_resample_global(G, P, mode):
    """vpf_estimate_resample (the ParticleFilter product path) over G gathered shard chunks: every rank's slots get
    the global oracle's ancestors and states bit for bit, the resample word drawn on the device equals SPEC S1's,
    T is exact, and the fp64 sums are the same bits for every G (and as vpf_shard_stats over the whole set)."""
    from vitparticlefiltertracker_amd.particle_filter import (chunk_words, compact_index, compact_view, global_view,
                                                                shard_range, shard_views)
    if G > P:
        pytest.skip("more ranks than particles")
    rng = np.random.default_rng(P + G)
    Q = rng.integers(0, 1 << 40, P, dtype=np.int64)
    if mode == "sparse":
        Q[rng.random(P) < 0.9] = 0
    if mode == "zero":
        Q[:] = 0
    if mode == "onehot":
        Q[:] = 0
        Q[P // 3] = 12345
    p = rng.uniform(0, 224, (3, P)).astype(np.float32)
    seed, frame = (1 << 40) + 17 * P, 9
    ref = pf.resample(Q, pf.resample_U(seed, frame))
    T_ref, sums_ref = pf.shard_stats(Q, p)
    n_max = -(-P // G)   # unequal shards (P = 7 over 2): chunks sized for the largest, compacted as ParticleFilter does
    cw = chunk_words(n_max)
    allc = torch.zeros(G * cw, dtype=torch.int32)
    for r in range(G):
        b, n = shard_range(P, G, r)
        Qv, pv = shard_views(allc[r * cw:(r + 1) * cw], n)
        Qv.copy_(torch.from_numpy(Q[b:b + n].copy()))
        pv.copy_(torch.from_numpy(p[:, b:b + n].copy()))
    allc = allc.to(DEV)
    view = (global_view(allc, G, n_max) if P % G == 0
            else compact_view(torch.index_select(allc, 0, compact_index(P, G).to(DEV)), P))
    # the world-1 form ParticleFilter passes: its own Q and particle arrays, one shard of P
    Qd, pd = torch.from_numpy(Q).to(DEV), torch.from_numpy(p).to(DEV)
    view1 = (Qd, P, pd.view(-1), P, 3 * P, P)
    cdf = torch.empty(P, device=DEV, dtype=torch.int64)
    stats1 = torch.empty(4, device=DEV, dtype=torch.int64)
    anc1 = torch.empty(P, device=DEV, dtype=torch.int32)
    st1 = torch.empty(3, P, device=DEV)
    vpf().estimate_resample(*view1, P, seed, frame, 0, P, anc1, st1, cdf, stats1)
    assert np.array_equal(anc1.cpu().numpy(), ref)
    assert np.array_equal(st1.cpu().numpy(), p[:, ref])
    s1 = stats1.cpu()
    assert int(s1[0]) == T_ref
    if T_ref:
        np.testing.assert_allclose(s1[1:].view(torch.float64).numpy(), sums_ref, rtol=1e-13)
        To = torch.empty(1, device=DEV, dtype=torch.int64)
        So = torch.empty(3, device=DEV, dtype=torch.float64)
        vpf().shard_stats(Qd, pd, To, So)
        assert torch.equal(s1[1:].view(torch.float64), So.cpu())
    else:   # uniform fallback: the plain sums (estimate = sum / P)
        np.testing.assert_allclose(s1[1:].view(torch.float64).numpy(), p.astype(np.float64).sum(axis=1), rtol=1e-13)
    for r in range(G):
        b, n = shard_range(P, G, r)
        anc = torch.full((n,), -1, device=DEV, dtype=torch.int32)
        st = torch.empty(3, n, device=DEV)
        stats = torch.empty(4, device=DEV, dtype=torch.int64)
        vpf().estimate_resample(*view, P, seed, frame, b, b + n, anc, st, cdf, stats)
        assert np.array_equal(anc.cpu().numpy(), ref[b:b + n]), f"shard {r}: ancestors"
        assert np.array_equal(st.cpu().numpy().view(np.uint32), p[:, ref[b:b + n]].view(np.uint32))
        assert torch.equal(stats.cpu(), s1), f"shard {r}: statistics bits depend on G"


@pytest.mark.parametrize("M,N,K,S", [(1, 768, 768, 3), (37, 768, 3072, 12), (512, 768, 3072, 12), (700, 3072, 768, 3),
                                     (300, 192, 192, 1), (256, 1024, 4096, 16)])
@pytest.mark.parametrize("epi", [0, 1, 2, 4, 5])
def test_gemm_splitk(M, N, K, S, epi):
    """vpf_gemm_bf16_splitk (the last block's CLS-row GEMMs) vs an fp64 reference of the same epilogue, on
    row-strided views (the CLS rows of a token tensor); with the residual in place and its statistics planes; and
    a row's bits independent of the call's row count (the first rows of an M-row call equal a 1-row call)."""
    torch.manual_seed(M + N + K + epi)
    stride = 3 * max(N, K)                          # rows strided like the CLS rows of [n][N_tok][D]
    Abuf = torch.randn(M, stride, device=DEV).to(torch.bfloat16)
    A = Abuf[:, :K]
    W = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    bias = 0.1 * torch.randn(N, device=DEV)
    ws = torch.empty(S * M * N, device=DEV)
    st = colsum = None
    Rbuf = torch.randn(M, stride, device=DEV).to(torch.bfloat16)
    out = Rbuf[:, :N] if epi == 2 else torch.empty(M, stride, device=DEV, dtype=torch.bfloat16)[:, :N]
    R0 = Rbuf[:, :N].clone()
    acc = A.double() @ W.double().t()
    if epi in (4, 5):
        st = torch.stack([torch.randn(M, device=DEV) * 0.1, 1.0 + torch.rand(M, device=DEV)], 1).contiguous()
        colsum = W.float().sum(1)
        acc = st[:, 1:].double() * acc - (st[:, 1:] * st[:, :1]).double() * colsum.double() + bias.double()
    else:
        acc = acc + bias.double()
    planes = torch.full((N // 64, M, 2), 7.0, device=DEV) if epi == 2 and N % 64 == 0 else None
    vpf().gemm_splitk_(A, W, bias, out if epi == 2 else None, st, colsum, epi, S, out, planes, ws)
    if epi in (1, 5):
        ref = Fn.gelu(acc)
    elif epi == 2:
        ref = acc.to(torch.bfloat16).double() + R0.double()
    else:
        ref = acc
    torch.testing.assert_close(out.double(), ref, rtol=1.6e-2, atol=1.5e-2)
    if planes is not None:
        torch.testing.assert_close(planes.double(), _planes_ref(out, N // 64), rtol=1e-4, atol=1e-3)
    if epi != 2:   # row invariance: the first row alone gives the same bits
        one = torch.empty(1, N, device=DEV, dtype=torch.bfloat16)
        vpf().gemm_splitk_(A[:1], W, bias, None, None if st is None else st[:1].contiguous(), colsum, epi, S, one,
                           None, ws)
        assert torch.equal(one[0], out[0])


def test_gemm_splitk_rejects_bad_split():
    A = torch.zeros(4, 768, device=DEV, dtype=torch.bfloat16)
    W = torch.zeros(768, 768, device=DEV, dtype=torch.bfloat16)
    out = torch.empty(4, 768, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(Exception):   # 768 is not a multiple of 64 * 5
        vpf().gemm_splitk_(A, W, torch.zeros(768, device=DEV), None, None, None, 0, 5, out, None,
                           torch.empty(5 * 4 * 768, device=DEV))


def test_particle_filter_api_matches_oracle():
    """The ParticleFilter surface driven directly, 1000 particles over 5 frames: predict() equals the
    oracle's S2 walk bit for bit; update(features, template) gives Q = weights_to_Q of the kernel's cosine (itself
    within 1e-5 of numpy's); estimate() equals the oracle's S6 estimate; resample() returns the oracle's S7
    ancestors and the particles become their states; `particles` (and its alias `states`) is the [P][3] view of the SoA
    storage `particles_soa`."""
    from vitparticlefiltertracker_amd.particle_filter import ParticleFilter
    P, D, seed = 1000, 192, 321
    std, srange = (3.0, 2.0, 0.03), (0.6, 1.8)
    f = ParticleFilter(P, (100.0, 90.0, 1.0), std, srange, seed, DEV, frame_size=(224, 224), lam=20.0, weight_bits=40)
    ref = np.empty((3, P), np.float32)
    ref[0], ref[1], ref[2] = 100.0, 90.0, 1.0
    rng = np.random.default_rng(5)
    t = rng.standard_normal(D).astype(np.float32)
    t /= np.linalg.norm(t)
    for k in range(1, 6):
        f.predict()
        pf.predict(ref, 0, seed, k, std, 224, 224, srange)
        assert np.array_equal(f.particles_soa.cpu().numpy().view(np.uint32), ref.view(np.uint32)), f"frame {k}: predict"
        assert f.states.shape == (P, 3) and torch.equal(f.states.cpu(), torch.from_numpy(ref.T.copy()))
        # a §8b-style caller: particles is [P, 3], so column 0 is every particle's x
        assert f.particles.shape == (P, 3)
        for c in range(3):
            assert np.array_equal(f.particles[:, c].cpu().numpy().view(np.uint32), ref[c].view(np.uint32))
        feat = (rng.standard_normal((P, D)) + 2.0 * t).astype(np.float32)
        Q = f.update(torch.from_numpy(feat).to(DEV), torch.from_numpy(t).to(DEV)).cpu().numpy()
        sim = torch.empty(P, device=DEV)
        vpf().cosine_weight(torch.from_numpy(feat).to(DEV), torch.from_numpy(t).to(DEV), 20.0, 40,
                            torch.empty(P, device=DEV, dtype=torch.int64), sim)
        s = sim.cpu().numpy()
        cos = feat.astype(np.float64) @ t / np.linalg.norm(feat.astype(np.float64), axis=1)
        np.testing.assert_allclose(s, cos, atol=1e-5)
        assert np.array_equal(Q, pf.weights_to_Q(s, 20.0, 40)), f"frame {k}: Q"
        est = f.estimate()
        np.testing.assert_allclose(est, pf.estimate(Q, ref), rtol=1e-12)
        anc = f.resample().cpu().numpy()
        anc_ref = pf.resample(Q, pf.resample_U(seed, k))
        assert np.array_equal(anc, anc_ref), f"frame {k}: ancestors"
        ref = np.ascontiguousarray(ref[:, anc_ref])
        assert np.array_equal(f.particles_soa.cpu().numpy().view(np.uint32), ref.view(np.uint32)), f"frame {k}: states"
