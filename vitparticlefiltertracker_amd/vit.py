"""ViT feature extractor on the HIP path (the reference's "Vision Transformer (ViT)
... feature extraction", /root/reference/README.md:7).

`ViTEngine` holds the device weights and every activation buffer for a fixed particle batch and runs one
frame's forward as a fixed chain of `torch.ops.vpf.*` launches on the current HIP stream:

    crop+im2col -> patch GEMM (+bias +pos, scattered into token rows) -> CLS rows
    L x [ LN1 -> QKV GEMM(+bias) -> attention -> proj GEMM(+bias +residual, in place on h)
          LN2 -> FC1 GEMM(+bias +GELU) -> FC2 GEMM(+bias +residual, in place on h) ]
    final LN of the CLS rows -> cosine to the template -> int64 fixed-point weights Q

Because every buffer is preallocated and no launch synchronises, the chain is captured once into a HIP
graph (`torch.cuda.CUDAGraph`, which is a hipGraph on ROCm) and replayed per frame (`capture=True`).

HBM layout (bf16 mode, P particles, N tokens, D width, F MLP width):
  h   [P][N][D]   residual stream (bf16)          x   [P][N][D]   LN output / attention output
  qkv [P][N][3D]  (3, heads, 64) column order      hid [P][N][F]   GELU(FC1) (also hosts the im2col patches)
Weights are [out][in] (K-contiguous rows) bf16 with fp32 biases / LayerNorm affines / cls / pos.

fp8 mode (model.dtype = "fp8", BASELINE.json configs[4]): the QKV, proj, FC1 and FC2 GEMMs run on
block-scaled MFMA (vpf_gemm_mx8) with MX-fp8 weights (quantised once from the LN-folded bf16 weights) and
MX-fp8 activations written by the producing kernels:
  h8   MX8 copy of h   (patch embed / proj / FC2 epilogues; CLS rows by vpf_quantize_mx8) -> QKV, FC1 A operand
  x8   MX8 attention output (vpf_attention_bf16_mx8; shares hid8's storage)              -> proj A operand
  hid8 MX8 GELU(FC1)   (FC1 epilogue, no bf16 copy)                                      -> FC2 A operand
The residual stream h, qkv and the attention arithmetic stay bf16, as does the last block's CLS-row tail (and,
for N > 256, the attention output and proj).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from . import _lib
from . import ops  # registers torch.ops.vpf; rgba_workspace
from .config import ViTArch

vpf = torch.ops.vpf


def norm_affine(mean, std):
    """SPEC S3 per-channel affine {a0,a1,a2,b0,b1,b2} in fp32 (same rounding as the oracle)."""
    one = torch.tensor(1.0, dtype=torch.float32)
    inv255 = one / torch.tensor(255.0, dtype=torch.float32)
    a, b = [], []
    for c in range(3):
        inv_std = one / torch.tensor(float(std[c]), dtype=torch.float32)
        a.append(float((inv255 * inv_std).item()))
        b.append(float((-torch.tensor(float(mean[c]), dtype=torch.float32) * inv_std).item()))
    return a + b


def _splits(K: int) -> int:
    """K-chunks of the split-K CLS-row fc2: ~768 deep each (the largest s <= K / 768 with K % (64 s) == 0). Deeper
    chunks would leave the 512-row case latency-bound, shallower ones cost more partial-plane traffic than they save
    at 4096-8192 rows (profiles/r2_gemm_lab/cls_splitk_depth.txt)."""
    s = max(1, K // 768)
    while K % (64 * s):
        s -= 1
    return s


class KernelTimer:
    """HIP-event timing of individual launches on the current stream (eager mode only; bench.py)."""

    def __init__(self):
        self.pending = []     # (name, start, end)

    def __call__(self, name, fn, *args):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        fn(*args)
        e.record()
        self.pending.append((name, s, e))

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for name, s, e in self.pending:
            d = out.setdefault(name, [0, 0.0])
            d[0] += 1
            d[1] += s.elapsed_time(e)
        return {k: {"launches": v[0], "total_ms": v[1], "avg_ms": v[1] / v[0]} for k, v in out.items()}


def _run(timer, name, fn, *args):
    if timer is None:
        fn(*args)
    else:
        timer(name, fn, *args)


class ViTEngine:
    def __init__(self, arch: ViTArch, weights: Dict[str, torch.Tensor], dtype: str, device, batch: int,
                 mean=(0.5, 0.5, 0.5), std=(0.5, 0.5, 0.5), cls_fused: bool = True, cls_splitk: bool = True):
        """`cls_fused` / `cls_splitk` (default on, the product): the last block's folded CLS attention and its split-K
        CLS-row fc2. Off selects the K / V GEMM + attention path and the one-pass fc2 they replace (tests, A/B); no
        environment variable changes what the engine runs."""
        if not torch.cuda.is_available():
            raise _lib.VPFError("ViTEngine needs a HIP device (the product path has no CPU fallback)")
        _lib.lib()  # fail loudly now if libvpf.so is missing
        self.arch = arch
        self.device = torch.device(device)
        if dtype not in ("bf16", "fp8", "fp32"):
            raise ValueError(f"dtype {dtype!r}: bf16 | fp8 | fp32")
        self.fp8 = dtype == "fp8"
        self.dt = torch.float32 if dtype == "fp32" else torch.bfloat16
        if self.fp8 and (arch.dim % 128 or arch.mlp % 128):
            raise ValueError(f"fp8 mode needs D and the MLP width divisible by 128 (MX8 K-tiles); {arch.name} has "
                             f"D = {arch.dim}")
        self.batch = int(batch)
        self.norm_ab = norm_affine(mean, std)
        A = arch
        D, F, N = A.dim, A.mlp, A.tokens
        dev, dt = self.device, self.dt

        def mat(t):
            return t.to(dev, dt).contiguous()

        def f32(t):
            return t.to(dev, torch.float32).contiguous()

        wpe = weights["patch_embed.weight"].reshape(D, A.patch_k)
        wpe_p = torch.zeros(D, A.patch_kp)
        wpe_p[:, :A.patch_k] = wpe
        self.w_pe = mat(wpe_p)
        self.b_pe = f32(weights["patch_embed.bias"])
        self.cls = f32(weights["cls_token"])
        self.pos = f32(weights["pos_embed"])
        # bf16 product mode folds each pre-GEMM LayerNorm into the GEMM (vpf_gemm_bf16 EPI_LN*):
        # W' = W diag(gamma) (bf16), colsum = row sums of the rounded W', b' = b + W beta; the GEMM then
        # reads the raw residual stream and the epilogue applies the per-row (mean, rstd). fp32 parity mode
        # keeps the explicit LayerNorm kernel (the oracle's operation order).
        self.fold_ln = self.dt == torch.bfloat16

        def folded(wname, bname, gname, bename):
            Wf = weights[wname].float()
            g, be = weights[gname].float(), weights[bename].float()
            Wg = (Wf * g.unsqueeze(0)).to(dt)
            colsum = Wg.float().sum(dim=1)
            bias = weights[bname].float() + Wf @ be
            return Wg.to(dev).contiguous(), f32(bias), f32(colsum)

        self.layers = []
        for l in range(A.depth):
            p = f"blocks.{l}."
            L = {
                "n1g": f32(weights[p + "norm1.weight"]), "n1b": f32(weights[p + "norm1.bias"]),
                "wproj": mat(weights[p + "attn.proj.weight"]), "bproj": f32(weights[p + "attn.proj.bias"]),
                "n2g": f32(weights[p + "norm2.weight"]), "n2b": f32(weights[p + "norm2.bias"]),
                "wfc2": mat(weights[p + "mlp.fc2.weight"]), "bfc2": f32(weights[p + "mlp.fc2.bias"]),
            }
            if self.fold_ln:
                L["wqkv"], L["bqkv"], L["cqkv"] = folded(p + "attn.qkv.weight", p + "attn.qkv.bias",
                                                         p + "norm1.weight", p + "norm1.bias")
                L["wfc1"], L["bfc1"], L["cfc1"] = folded(p + "mlp.fc1.weight", p + "mlp.fc1.bias",
                                                         p + "norm2.weight", p + "norm2.bias")
            else:
                L["wqkv"], L["bqkv"] = mat(weights[p + "attn.qkv.weight"]), f32(weights[p + "attn.qkv.bias"])
                L["wfc1"], L["bfc1"] = mat(weights[p + "mlp.fc1.weight"]), f32(weights[p + "mlp.fc1.bias"])
            if self.fp8:
                # MX8 copies of the three GEMMs that run on block-scaled MFMA; LN-fold colsums of the
                # dequantised W' so the fold's algebra holds exactly for the weights the MFMA multiplies
                for key in ("wqkv", "wproj", "wfc1", "wfc2"):
                    q, sc = ops.mx8_empty(L[key].shape[0], L[key].shape[1], dev)
                    vpf.quantize_mx8_(L[key], 1, q, sc)
                    L[key + "8"] = (q, sc)
                for key, ck in (("wqkv", "cqkv"), ("wfc1", "cfc1")):
                    L[ck + "8"] = ops.mx8_dequantize(*L[key + "8"]).sum(dim=1).contiguous()
                q, sc = L["wqkv8"]
                L["wkv8"] = (q[D:], sc[:, D:].contiguous())        # the last block's K | V rows (64-row bricks)
            self.layers.append(L)
        self.ng = f32(weights["norm.weight"])
        self.nb = f32(weights["norm.bias"])
        # the last block's CLS attention without K / V (vpf_cls_attn_fold_bf16): LN-folded bf16 with statistics
        # planes, head dim 64, 6, 12 or 16 heads, N <= 640. The per-head algebra:
        #   G[p][h D + i] = sum_{k in head h} q[p][k] W'_k[k][i]   block-diagonal GEMM (W_G[h D + i][k] = W'_k[k][i])
        #   x[p][64 h + d] = sum_i W'_v[64 h + d][i] U[p][h D + i] + b'_v[64 h + d]: one dense GEMM of the (p, h)
        #   rows of U against W'_v, then the diagonal blocks gathered (vpf_head_gather_bf16)
        # cls_fused=False keeps the K / V GEMM + attention path (A/B, tests).
        H = A.heads
        self.cls_fused = bool(cls_fused) and self.fold_ln and H in (6, 12, 16) and D == 64 * H and N <= 640
        self.cls_splitk = bool(cls_splitk)
        if self.cls_fused:
            L = self.layers[-1]
            Wk = L["wqkv"][D:2 * D].float()
            wg = torch.zeros(H * D, D, device=dev, dtype=torch.float32)
            for h in range(H):
                c = slice(64 * h, 64 * h + 64)
                wg[h * D:(h + 1) * D, c] = Wk[c, :].t()
            self.w_clsG = wg.to(dt).contiguous()
            self.b_clsG = torch.zeros(H * D, device=dev, dtype=torch.float32)
        self._alloc(self.batch)
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.timer: Optional[KernelTimer] = None

    # ------------------------------------------------------------------ buffers
    def _alloc(self, n: int) -> None:
        A, dev, dt = self.arch, self.device, self.dt
        D, F, N = A.dim, A.mlp, A.tokens
        self.h = torch.empty(n, N, D, device=dev, dtype=dt)
        self.x = torch.empty(n, N, D, device=dev, dtype=dt)
        self.qkv = torch.empty(n, N, 3 * D, device=dev, dtype=dt)
        # hid: the bf16 MLP hidden of every token row; in fp8 mode FC1 writes MX8 (hid8) and the bf16 hidden holds only
        # the last block's CLS rows, so it is sized for those (configs[4]: 7.4 GB less per 8192 particles). It also
        # hosts the im2col patches (free until the first FC1).
        hid_rows = n if self.fp8 else n * N
        hid_elems = max(hid_rows * F, n * A.n_patches * A.patch_kp)
        self.hid_flat = torch.empty(hid_elems, device=dev, dtype=dt)
        self.hid = self.hid_flat[: hid_rows * F].view(hid_rows, F)
        self.patches = self.hid_flat[: n * A.n_patches * A.patch_kp].view(n * A.n_patches, A.patch_kp)
        self.stats = torch.empty(n * N, 2, device=dev, dtype=torch.float32)
        # bf16 fold mode: residual-stream statistics planes written by the GEMMs that produce h (patch embed,
        # proj, fc2) and read by the LN-folded GEMMs (qkv, fc1): [P][rows][2] {sum, sumsq} per 64-column block.
        # P <= 16 (the consumer's LDS copy, ViT-L's D = 1024); wider models keep the row_stats pass.
        self.parts = (D + 63) // 64
        self.use_planes = self.fold_ln and self.parts <= 16
        self.planes_flat = torch.empty(self.parts * n * N * 2, device=dev, dtype=torch.float32)
        self.planes_cls_flat = torch.empty(self.parts * n * 2, device=dev, dtype=torch.float32)
        if self.fp8:
            self.h8 = ops.mx8_empty(n * N, D, dev)
            self.hid8 = ops.mx8_empty(n * N, F, dev)
        if self.cls_fused:
            self.clsG = torch.empty(n, A.heads * D, device=dev, dtype=dt)
            self.clsU = torch.empty(n, A.heads * D, device=dev, dtype=dt)
        if self.fold_ln:   # split-K partial planes of the last block's CLS-row GEMMs (q, proj, fc2)
            self.splitk_ws = torch.empty(n * D * _splits(F), device=dev, dtype=torch.float32)
        self.Q = torch.empty(n, device=dev, dtype=torch.int64)
        self.feat = torch.empty(n, D, device=dev, dtype=torch.float32)
        self.sim = torch.empty(n, device=dev, dtype=torch.float32)

    # ------------------------------------------------------------------ forward pieces
    def embed(self, frame: torch.Tensor, particles: torch.Tensor, box_wh) -> None:
        A = self.arch
        n = particles.shape[1]
        patches = self.patches[: n * A.n_patches]
        T = self.timer
        hw = (int(frame.shape[0]), int(frame.shape[1]))
        if getattr(self, "_rgba_hw", None) != hw:          # workspace sized for this frame shape
            self.rgba = ops.rgba_workspace(hw, frame.device)
            self._rgba_hw = hw
        _run(T, "crop_patches", vpf.crop_patches, frame, self.rgba, particles, [float(box_wh[0]), float(box_wh[1])],
             A.img_size, A.patch, self.norm_ab, patches)
        self._embed_rest(n)

    def _embed_rest(self, n: int) -> None:
        """Patch GEMM (+ bias + position rows, CLS-offset token rows) and the CLS rows for the first n crops."""
        A = self.arch
        T = self.timer
        patches = self.patches[: n * A.n_patches]
        h = self.h[:n]
        pl = self.planes(n) if self.use_planes else None
        if self.fp8:
            N = A.tokens
            pl = pl if pl is not None else self.planes_flat[: self.parts * n * N * 2].view(self.parts, n * N, 2)
            h8q, h8s = self.h8
            _run(T, "gemm_patch", vpf.gemm_q8_, patches, self.w_pe, self.b_pe, None, self.pos, A.n_patches,
                 _lib.VPF_EPI_PATCH, h, pl, h8q, h8s)
            _run(T, "cls_rows", vpf.cls_rows_stats_, h, self.cls, self.pos, pl)
            _run(T, "cls_q8", vpf.quantize_mx8_, h.view(n, N * A.dim)[:, :A.dim], N, h8q, h8s)
        elif pl is not None:
            _run(T, "gemm_patch", vpf.gemm_stats_, patches, self.w_pe, self.b_pe, None, self.pos, A.n_patches,
                 _lib.VPF_EPI_PATCH, h, pl)
            _run(T, "cls_rows", vpf.cls_rows_stats_, h, self.cls, self.pos, pl)
        else:
            _run(T, "gemm_patch", vpf.gemm, patches, self.w_pe, self.b_pe, None, self.pos, A.n_patches, None, None,
                 _lib.VPF_EPI_PATCH, h)
            _run(T, "cls_rows", vpf.cls_rows_, h, self.cls, self.pos)

    def embed_many(self, frame: torch.Tensor, particle_sets, boxes) -> int:
        """Multi-object embed: particle set k (float32[3][n_k]) cropped with its own template box boxes[k] into
        consecutive patch rows, then one patch GEMM + CLS rows over all of them. Returns the total count."""
        A = self.arch
        n = sum(int(p.shape[1]) for p in particle_sets)
        assert n <= self.batch
        hw = (int(frame.shape[0]), int(frame.shape[1]))
        if getattr(self, "_rgba_hw", None) != hw:
            self.rgba = ops.rgba_workspace(hw, frame.device)
            self._rgba_hw = hw
        row = 0
        for parts, box in zip(particle_sets, boxes):
            k = int(parts.shape[1])
            _run(self.timer, "crop_patches", vpf.crop_patches, frame, self.rgba, parts, [float(box[0]), float(box[1])],
                 A.img_size, A.patch, self.norm_ab, self.patches[row * A.n_patches:(row + k) * A.n_patches])
            row += k
        self._embed_rest(n)
        return n

    def planes(self, n: int) -> torch.Tensor:
        """Statistics planes of h[:n] (plane stride n*N rows, as the producing GEMMs write them)."""
        N = self.arch.tokens
        return self.planes_flat[: self.parts * n * N * 2].view(self.parts, n * N, 2)

    def encoder(self, n: int) -> None:
        """L pre-norm blocks on h[:n]. The last block only needs the CLS rows after its attention (the
        final LN reads nothing else): its QKV GEMM computes K, V for every row but Q for the CLS rows only,
        its attention computes the CLS query only (q_rows = 1), and its proj / MLP run on the n strided CLS
        rows. With `cls_fused` (LN-folded bf16 / fp8, 6, 12 or 16 heads) K and V are never formed: the CLS query
        goes through W'_k per head (G), vpf_cls_attn_fold_bf16 reads the token rows once, and W'_v maps the
        result back (csrc/cls_attn.hip)."""
        A = self.arch
        D, N, F = A.dim, A.tokens, A.mlp
        T = self.timer
        h2 = self.h[:n].view(n * N, D)
        x2 = self.x[:n].view(n * N, D)
        qkv = self.qkv[:n]
        hid = self.hid[: n * N]
        st = self.stats[: n * N]
        hc = self.h[:n].view(n, N * D)[:, :D]       # CLS rows (row stride N*D)
        xc = self.x[:n].view(n, N * D)[:, :D]
        hidc = self.hid[:n]
        stc = self.stats[:n]
        BIAS, GELU, RES = _lib.VPF_EPI_BIAS, _lib.VPF_EPI_BIAS_GELU, _lib.VPF_EPI_BIAS_RESIDUAL
        LNE, LNG = _lib.VPF_EPI_LN, _lib.VPF_EPI_LN_GELU
        fold, planes = self.fold_ln, self.use_planes
        P, eps = self.parts, A.ln_eps
        pl = self.planes(n) if planes else None                # planes of h2 (written by embed / proj / fc2)
        ws = self.splitk_ws if fold else None
        sk = fold and self.cls_splitk                         # False: the one-pass kernel (A/B timing)

        def q_cls():
            """The CLS rows' LN-folded query (row statistics from the row_stats pass in stc)."""
            _run(T, "gemm_q_cls", vpf.gemm, hc, L["wqkv"][:D], L["bqkv"][:D], None, None, 0, stc, L["cqkv"][:D],
                 LNE, qc)
        plc = self.planes_cls_flat[: P * n * 2].view(P, n, 2)  # planes of the last block's CLS rows

        def ln_stats(x, st_rows, pln):
            """LayerNorm statistics of rows x for an LN-folded GEMM: the producer's planes combined into {mean, rstd} by
            one small pass (vpf_stats_combine: 8 B per plane and row), then the GEMM reads one {mean, rstd} plane. The
            result is bit-identical to the GEMM combining the planes itself, and faster, combine included (round 5,
            profiles/r5_lab/planes_combine_ab.txt): ViT-B QKV -1.8 %, FC1 -0.9 %; ViT-L QKV -4.0 %, FC1 -4.4 % (its 16
            planes exceed what the ping-pong kernel holds in LDS, so QKV / FC1 also leave kernel 1's wide form).
            Without planes (no fold or > 16 of them) a row_stats pass."""
            if planes:
                _run(T, "stats_combine", vpf.stats_combine_, pln, D, eps, st_rows)
                return st_rows, 0
            _run(T, "row_stats", vpf.row_stats, x, eps, st_rows)
            return st_rows, 0

        def residual_gemm(name, a, w, b, hh_, pln):
            """h += a w^T + b, also writing h's statistics planes when the consumers read them."""
            if planes and pln is not None:
                _run(T, name, vpf.gemm_stats_, a, w, b, hh_, None, 0, RES, hh_, pln)
            else:
                _run(T, name, vpf.gemm, a, w, b, hh_, None, 0, None, None, RES, hh_)

        q2 = qkv.view(n * N, 3 * D)
        kv2 = q2[:, D:]                                 # K | V columns of every row
        qc = qkv.view(n, N * 3 * D)[:, :D]             # Q columns of the CLS rows
        if self.fp8:
            h8q, h8s = self.h8
            h8q = h8q[: n * N]
            hq, hs = self.hid8
            hq8d = hq.view(-1)[: n * N * D].view(n * N, D)   # the attention's MX8 output (x8) shares hid8's storage
            hq = hq[: n * N]

            def ln_stats8(x):
                """LN statistics for an MX8 consumer: the planes combined into {mean, rstd} (as ln_stats: MX8 QKV -3.3 %
                in one process, bit-identical, profiles/r5_lab/planes_combine_ab.txt), else a row_stats pass."""
                if planes:
                    _run(T, "stats_combine", vpf.stats_combine_, pl, D, eps, st)
                    return st, 0
                _run(T, "row_stats", vpf.row_stats, x, eps, st)
                return st, 0
        for l, L in enumerate(self.layers):
            last = l == len(self.layers) - 1
            if self.fp8 and not last:
                s1, p1 = ln_stats8(h2)
                _run(T, "gemm_qkv", vpf.gemm_mx8, h8q, h8s, *L["wqkv8"], L["bqkv"], None, s1, L["cqkv8"], LNE, q2,
                     p1, eps)
                if N <= 256:   # attention writes MX8 (into hid8's storage, free until FC1) -> MX8 proj
                    x8q, x8s = hq8d, hs[: D // 128]
                    _run(T, "attention", vpf.attention_q8_, qkv, A.heads, x8q, x8s)
                    _run(T, "gemm_proj", vpf.gemm_mx8_res_, x8q, x8s, *L["wproj8"], L["bproj"], h2, pl, h8q, h8s)
                else:
                    _run(T, "attention", vpf.attention, qkv, A.heads, N, self.x[:n])
                    _run(T, "gemm_proj", vpf.gemm_q8_, x2, L["wproj"], L["bproj"], h2, None, 0, RES, h2, pl, h8q,
                         h8s)
                s2, p2 = ln_stats8(h2)
                _run(T, "gemm_fc1", vpf.gemm_mx8_q8_, h8q, h8s, *L["wfc18"], L["bfc1"], s2, L["cfc18"], LNG, hq, hs,
                     p2, eps)
                _run(T, "gemm_fc2", vpf.gemm_mx8_res_, hq, hs, *L["wfc28"], L["bfc2"], h2, pl, h8q, h8s)
                continue
            # the last block's attention reads only the CLS query: K, V for every row, Q for the CLS rows
            if fold:
                if not last:
                    s1, p1 = ln_stats(h2, st, pl)
                    _run(T, "gemm_qkv", vpf.gemm, h2, L["wqkv"], L["bqkv"], None, None, 0, s1, L["cqkv"], LNE, q2,
                         p1, eps)
                elif self.cls_fused:
                    # K, V never formed: the CLS query, G = W'_k^T q per head, the folded attention, then W'_v
                    _run(T, "row_stats", vpf.row_stats, hc, A.ln_eps, stc)     # the CLS rows' {mean, rstd}
                    q_cls()
                    G, U = self.clsG[:n], self.clsU[:n]
                    _run(T, "gemm_cls_g", vpf.gemm, qc, self.w_clsG, self.b_clsG, None, None, 0, None, None, BIAS, G)
                    _run(T, "attention_cls", vpf.cls_attn_fold_, self.h[:n], pl, eps, G, qc, L["bqkv"][D:2 * D],
                         A.heads, U)
                    Y = self.clsG[:n].view(n * A.heads, D)   # G's storage: G is consumed by attention_cls
                    _run(T, "gemm_cls_v", vpf.gemm, U.view(n * A.heads, D), L["wqkv"][2 * D:], L["bqkv"][2 * D:],
                         None, None, 0, None, None, BIAS, Y)
                    _run(T, "cls_v_gather", vpf.head_gather_, Y, A.heads, xc)
                elif self.fp8:
                    s8, p8 = ln_stats8(h2)
                    _run(T, "gemm_kv", vpf.gemm_mx8, h8q, h8s, *L["wkv8"], L["bqkv"][D:], None, s8, L["cqkv8"][D:],
                         LNE, kv2, p8, eps)
                    _run(T, "row_stats", vpf.row_stats, hc, A.ln_eps, stc)     # the CLS rows' {mean, rstd}
                    q_cls()
                else:
                    # the statistics only where a branch reads them: the CLS-fused and fp8 last blocks launch no
                    # full-row combine (23 combines per frame where 22 are read)
                    s1, p1 = ln_stats(h2, st, pl)
                    _run(T, "gemm_kv", vpf.gemm, h2, L["wqkv"][D:], L["bqkv"][D:], None, None, 0, s1, L["cqkv"][D:],
                         LNE, kv2, p1, eps)
                    _run(T, "row_stats", vpf.row_stats, hc, A.ln_eps, stc)     # the CLS rows' {mean, rstd}
                    q_cls()
            else:
                _run(T, "layernorm", vpf.layernorm, h2, L["n1g"], L["n1b"], A.ln_eps, x2)
                if not last:
                    _run(T, "gemm_qkv", vpf.gemm, x2, L["wqkv"], L["bqkv"], None, None, 0, None, None, BIAS, q2)
                else:
                    _run(T, "gemm_kv", vpf.gemm, x2, L["wqkv"][D:], L["bqkv"][D:], None, None, 0, None, None, BIAS,
                         kv2)
                    _run(T, "gemm_q_cls", vpf.gemm, xc, L["wqkv"][:D], L["bqkv"][:D], None, None, 0, None, None,
                         BIAS, qc)
            if not (last and fold and self.cls_fused):
                _run(T, "attention_cls" if last else "attention", vpf.attention, qkv, A.heads, 1 if last else N,
                     self.x[:n])
            hh, xx, hd_, ss, pp = (hc, xc, hidc, stc, plc) if last else (h2, x2, hid, st, pl)
            tag = "_cls" if last else ""
            if fold and last and sk:
                # the CLS rows (n of them): split-K fc2 (K = MLP: a few output tiles each running the whole K loop on
                # one CU otherwise; fixed split order, so a row's result does not depend on n). q / proj / fc1
                # (K = D) gain nothing from splitting at 512 rows and lose at 4096-8192 (the partial planes)
                residual_gemm("gemm_proj" + tag, xx, L["wproj"], L["bproj"], hh, pp)
                s2, p2 = ln_stats(hh, ss, pp)
                _run(T, "gemm_fc1" + tag, vpf.gemm, hh, L["wfc1"], L["bfc1"], None, None, 0, s2, L["cfc1"], LNG, hd_,
                     p2, eps)
                # the last block's output only feeds the final LayerNorm (cls_weight computes its own stats)
                _run(T, "gemm_fc2" + tag, vpf.gemm_splitk_, hd_, L["wfc2"], L["bfc2"], hh, None, None, RES, _splits(F),
                     hh, None, ws)
            elif fold:
                residual_gemm("gemm_proj" + tag, xx, L["wproj"], L["bproj"], hh, pp)
                s2, p2 = ln_stats(hh, ss, pp)
                _run(T, "gemm_fc1" + tag, vpf.gemm, hh, L["wfc1"], L["bfc1"], None, None, 0, s2, L["cfc1"], LNG, hd_,
                     p2, eps)
                # the last block's output only feeds the final LayerNorm (cls_weight computes its own stats)
                residual_gemm("gemm_fc2" + tag, hd_, L["wfc2"], L["bfc2"], hh, None if last else pl)
            else:
                _run(T, "gemm_proj" + tag, vpf.gemm, xx, L["wproj"], L["bproj"], hh, None, 0, None, None, RES, hh)
                _run(T, "layernorm", vpf.layernorm, hh, L["n2g"], L["n2b"], A.ln_eps, xx)
                _run(T, "gemm_fc1" + tag, vpf.gemm, xx, L["wfc1"], L["bfc1"], None, None, 0, None, None, GELU, hd_)
                _run(T, "gemm_fc2" + tag, vpf.gemm, hd_, L["wfc2"], L["bfc2"], hh, None, 0, None, None, RES, hh)

    def weights_from_tokens(self, n: int, tmpl: torch.Tensor, lam: float, bits: int, want_feat: bool = False,
                            row0: int = 0):
        r = slice(row0, row0 + n)
        _run(self.timer, "cls_weight", vpf.cls_weight, self.h[r], self.ng, self.nb, self.arch.ln_eps, tmpl,
             float(lam), int(bits), self.Q[r], self.feat[r] if want_feat else None, self.sim[r])
        return self.Q[r]

    def features(self, frame: torch.Tensor, particles: torch.Tensor, box_wh) -> torch.Tensor:
        """LN'd CLS features [n][D] fp32 (template init, tests)."""
        n = particles.shape[1]
        assert n <= self.batch
        self.embed(frame, particles, box_wh)
        self.encoder(n)
        dummy_t = torch.zeros(self.arch.dim, device=self.device, dtype=torch.float32)
        vpf.cls_weight(self.h[:n], self.ng, self.nb, self.arch.ln_eps, dummy_t, 0.0, 0, self.Q[:n], self.feat[:n],
                       None)
        return self.feat[:n]

    def features_many(self, frame: torch.Tensor, particle_sets, boxes) -> torch.Tensor:
        """LN'd CLS features [n][D] fp32 of several particle sets, set k cropped with its own box boxes[k] (the
        multi-object template update); rows in set order. A crop's features do not depend on the batch."""
        n = self.embed_many(frame, particle_sets, boxes)
        self.encoder(n)
        dummy_t = torch.zeros(self.arch.dim, device=self.device, dtype=torch.float32)
        vpf.cls_weight(self.h[:n], self.ng, self.nb, self.arch.ln_eps, dummy_t, 0.0, 0, self.Q[:n], self.feat[:n],
                       None)
        return self.feat[:n]

    def forward_weights(self, frame, particles, box_wh, tmpl, lam, bits, want_feat: bool = False):
        n = particles.shape[1]
        assert n <= self.batch
        self.embed(frame, particles, box_wh)
        self.encoder(n)
        return self.weights_from_tokens(n, tmpl, lam, bits, want_feat)
