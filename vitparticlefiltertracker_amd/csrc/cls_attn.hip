// Last encoder block, CLS query only, without materialising K and V (SURVEY.md §8a H6 + H9; the last block's
// outputs other than the CLS row feed nothing).
//
// With the LayerNorm folded as everywhere else (W' = W diag(gamma), b' = b + W beta, LNraw_j = (h_j - mean_j)
// rstd_j), the CLS query's attention in head h is
//   s_hj = q_h . k_hj = LNraw_j . G_h + c0_h,    G_h = W'_k,h^T q_h  (a D-vector),  c0_h = q_h . b'_k,h
//   o_h  = sum_j p_hj v_hj = W'_v,h U_h + b'_v,h,   U_h = sum_j p_hj LNraw_j,   p_h = softmax_j(s_h * scale)
// so the K / V GEMMs over all N tokens (2 x 2 N D^2 flops per particle) become one D-long dot and one D-long
// axpy per (token, head): this kernel. G comes from a block-diagonal GEMM of the CLS queries; o from one dense GEMM
// of the (particle, head) rows of U against W'_v (bias b'_v) whose diagonal blocks k_head_gather copies out (vit.py).
//
// One 256-thread workgroup (4 waves) per particle; the particle's N token rows stream through LDS once, in
// chunks of 16 rows (double-buffered, register-staged: chunk c+2 is loaded while chunk c is consumed), and
// both products run on MFMA against the raw bf16 rows, the LayerNorm applied algebraically per row:
//   scores  S[t][h] = rstd_t (h_t . G_h - mean_t sum(G_h)) + c0_h       v_mfma_f32_16x16x32_bf16, rows = tokens,
//           each wave a quarter of the D columns (its G slice resident: H/2 x 4 VGPRs), partials summed in LDS;
//   softmax online over the chunks per head (running max with lazy rescale, as attention.hip), weights
//           w_th = p_th rstd_t rounded to bf16, plus corr_h = sum_t w_th mean_t from the SAME rounded weights,
//           so U_h = (sum_t w_th h_t - corr_h) / l_h = sum_t w_th (h_t - mean_t) / l_h exactly;
//   U^T[dims][heads] += H_chunk^T W^T                                 v_mfma_f32_16x16x16_bf16, A operand by
//           the hardware-transposed LDS read (ds_read_b64_tr_b16), each wave H 16-dim tiles of its quarter.
// LDS chunk image: 16 rows of 2D bytes, 16-byte column chunk c of row r stored at c ^ (r & 15) (row reads of the
// score operand conflict-free; the transposed reads 2-way). HBM traffic = the token rows once + planes + G.
#include "vpf_common.h"
#include "../../include/vpf.h"

using namespace vpf;

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int NMAX = 640;   // tokens (ViT-L/14 @ 336: 577)
constexpr int CH = 16;   // token rows per chunk

__device__ __forceinline__ bf16x4 lds_tr(const char* base, int off) {
    typedef __attribute__((address_space(3))) bf16x4 lds_v4;
    const lds_v4* q = reinterpret_cast<const lds_v4*>((__attribute__((address_space(3))) const char*)((size_t)base) + off);
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<lds_v4*>(q));
}

template <int H>
__global__ __launch_bounds__(256) void k_cls_attn_fold(const bf16_t* __restrict__ tok, int N,
                                                       const float* __restrict__ planes, int64_t plane_rows,
                                                       float eps, const bf16_t* __restrict__ G, int64_t ldg,
                                                       const bf16_t* __restrict__ q, int64_t ldq,
                                                       const float* __restrict__ bk, float scale_log2,
                                                       bf16_t* __restrict__ out, int64_t ldo) {
    constexpr int D = 64 * H;
    constexpr int ROWB = 2 * D;           // bytes per row
    constexpr int RC = D / 8;             // 16-byte chunks per row
    constexpr int QD = D / 4;             // columns per wave
    constexpr int KS = QD / 32;           // score k-steps per wave (H / 2)
    constexpr int UT = QD / 16;           // U tiles per wave (H)
    constexpr int PIECES = CH * RC / 256; // staging chunks per thread (H / 2)
    static_assert(RC % 16 == 0 && CH * RC % 256 == 0, "layout");
    __shared__ __attribute__((aligned(16))) char img[2][CH * ROWB];
    __shared__ float sp[4][CH][16];
    __shared__ __attribute__((aligned(8))) bf16_t wl[16][CH];   // [head][token] bf16 weights (B operand)
    __shared__ float alpha_s[16];
    __shared__ float2 rs[NMAX];
    __shared__ float c0s[16], gsum[16], lfin[16], cfin[16];

    const int p = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int g = lane >> 4, li = lane & 15;
    const bf16_t* trow0 = tok + (int64_t)p * N * D;
    const bf16_t* Gp = G + (int64_t)p * ldg;
    const int nc = (N + CH - 1) / CH;

    // staging registers: chunk rows -> LDS image
    uint4 stg[PIECES];
    auto load_chunk = [&](int c) {
#pragma unroll
        for (int k = 0; k < PIECES; ++k) {
            const int piece = tid + 256 * k, r = piece / RC, col = piece % RC;
            const int t = c * CH + r;
            stg[k] = t < N ? *reinterpret_cast<const uint4*>(trow0 + (int64_t)t * D + col * 8) : make_uint4(0, 0, 0, 0);
        }
    };
    auto store_chunk = [&](int b) {
#pragma unroll
        for (int k = 0; k < PIECES; ++k) {
            const int piece = tid + 256 * k, r = piece / RC, col = piece % RC;
            *reinterpret_cast<uint4*>(img[b] + r * ROWB + ((col ^ (r & 15)) << 4)) = stg[k];
        }
    };
    load_chunk(0);

    // prologue: row statistics from the planes, c0_h = q_h . bk_h, sum(G_h), this wave's G slice
    for (int j = tid; j < N; j += 256) {
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int t = 0; t < H; ++t) {
            const float2 st = *reinterpret_cast<const float2*>(planes + ((int64_t)t * plane_rows + (int64_t)p * N + j) * 2);
            s1 += st.x;
            s2 += st.y;
        }
        const float mean = s1 * (1.0f / D);
        rs[j] = make_float2(mean, __builtin_amdgcn_rsqf(fmaxf(s2 * (1.0f / D) - mean * mean, 0.f) + eps));
    }
    for (int h = wid; h < H; h += 4) {
        float a = bf2f(q[(int64_t)p * ldq + h * 64 + lane]) * bk[h * 64 + lane];
        float gs = 0.f;
        const uint32_t* gr = reinterpret_cast<const uint32_t*>(Gp + (int64_t)h * D) + lane * (H / 2);
#pragma unroll
        for (int e = 0; e < H / 2; ++e) {
            const uint32_t w = gr[e];
            gs += bf2f((bf16_t)(w & 0xffff)) + bf2f((bf16_t)(w >> 16));
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            a += __shfl_xor(a, o, 64);
            gs += __shfl_xor(gs, o, 64);
        }
        if (lane == 0) {
            c0s[h] = a;
            gsum[h] = gs;
        }
    }
    bf16x8 gf[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (li < H) v = *reinterpret_cast<const uint4*>(Gp + (int64_t)li * D + QD * wid + 32 * ks + 8 * g);
        gf[ks] = __builtin_bit_cast(bf16x8, v);
    }
    store_chunk(0);
    if (nc > 1) load_chunk(1);
    __syncthreads();

    f32x4 u[UT];
#pragma unroll
    for (int t = 0; t < UT; ++t) u[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    // softmax state of head ch = tid >> 4 (one 16-lane group per head; heads >= H stay empty)
    const int ch = tid >> 4, ct = tid & 15;
    float m = -INFINITY, l = 0.f, corr = 0.f;

    for (int c = 0; c < nc; ++c) {
        const char* buf = img[c & 1];
        // ---- scores: S[token][head] partial over this wave's columns ----
        f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int col = (QD / 8) * wid + 4 * ks + g;
            const bf16x8 a = *reinterpret_cast<const bf16x8*>(buf + li * ROWB + ((col ^ li) << 4));
            s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, gf[ks], s, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) sp[wid][4 * g + i][li] = s[i];
        __syncthreads();
        // ---- online softmax of this chunk (thread = (head ch, token ct)) ----
        {
            const int t = c * CH + ct;
            float sc = -INFINITY;
            float2 mr = make_float2(0.f, 0.f);
            if (ch < H && t < N) {
                mr = rs[t];
                const float dot = sp[0][ct][ch] + sp[1][ct][ch] + sp[2][ct][ch] + sp[3][ct][ch];
                sc = (mr.y * (dot - mr.x * gsum[ch]) + c0s[ch]) * scale_log2;
            }
            float cm = sc;
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) cm = fmaxf(cm, __shfl_xor(cm, o, 64));
            // lazy rescale: the reference max only moves when the chunk max exceeds it by more than 8 (exp2 domain)
            float alpha = 1.f;
            if (cm > m + 8.f) {
                alpha = m == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m - cm);
                m = cm;
            }
            const float pr = sc == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(sc - m);
            const bf16_t wb = f2bf(pr * mr.y);
            float ps = pr, cs = bf2f(wb) * mr.x;
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) {
                ps += __shfl_xor(ps, o, 64);
                cs += __shfl_xor(cs, o, 64);
            }
            l = l * alpha + ps;
            corr = corr * alpha + cs;
            wl[ch][ct] = wb;
            if (ct == 0) alpha_s[ch] = alpha;
        }
        // ---- stage chunk c+1 (its buffer was last read before this iteration's first barrier) ----
        if (c + 1 < nc) store_chunk((c + 1) & 1);
        if (c + 2 < nc) load_chunk(c + 2);
        __syncthreads();
        // ---- U^T[dims][heads] = alpha U^T + H_chunk^T W^T ----
        const float al = alpha_s[li];
        if (__builtin_expect(__any(al != 1.f), 0)) {
#pragma unroll
            for (int t = 0; t < UT; ++t) u[t] *= al;
        }
        const bf16x4 wf = *reinterpret_cast<const bf16x4*>(&wl[li][4 * g]);
        const int rq = 4 * g + (li >> 2), pp = li & 3;
#pragma unroll
        for (int t = 0; t < UT; ++t) {
            const int c0 = (QD / 8) * wid + 2 * t + (pp >> 1);
            const bf16x4 a = lds_tr(buf, rq * ROWB + ((c0 ^ rq) << 4) + (pp & 1) * 8);
            u[t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, wf, u[t], 0, 0, 0);
        }
    }
    if (ct == 0 && ch < 16) {
        lfin[ch] = l;
        cfin[ch] = corr;
    }
    __syncthreads();
    // out[head][dim] = (U - corr) / l: lane (head li, dims 4g .. 4g+3 of each tile)
    if (li < H) {
        const float inv = 1.0f / lfin[li], cr = cfin[li];
        bf16_t* orow = out + (int64_t)p * ldo + (int64_t)li * D + QD * wid + 4 * g;
#pragma unroll
        for (int t = 0; t < UT; ++t)
            *reinterpret_cast<uint2*>(orow + 16 * t) =
                make_uint2(pack_bf2((u[t][0] - cr) * inv, (u[t][1] - cr) * inv),
                           pack_bf2((u[t][2] - cr) * inv, (u[t][3] - cr) * inv));
    }
}

// out[p][h hd + d] = Y[p H + h][h hd + d]: the diagonal blocks of the dense per-(particle, head) V projection.
__global__ __launch_bounds__(256) void k_head_gather(const uint4* __restrict__ Y, int64_t n, int H, int hd8,
                                                     uint4* __restrict__ out, int64_t ldo8) {
    const int64_t D8 = (int64_t)H * hd8;   // 16-B pieces per row
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * D8) return;
    const int64_t p = i / D8;
    const int c = (int)(i - p * D8), h = c / hd8;
    out[p * ldo8 + c] = Y[(p * H + h) * D8 + c];
}

}  // namespace

VPF_API int vpf_head_gather_bf16(const uint16_t* Y, int64_t n, int H, int hd, uint16_t* out, int64_t ldo,
                                 void* stream) {
    if (n < 0 || H <= 0 || hd <= 0 || hd % 8 != 0 || ldo < (int64_t)H * hd || ldo % 8 != 0 || !Y || !out ||
        ((uintptr_t)Y & 15) || ((uintptr_t)out & 15))
        return VPF_ERR_ARG;
    if (n == 0) return 0;
    const int64_t work = n * H * (hd / 8);
    hipLaunchKernelGGL(k_head_gather, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const uint4*>(Y), n, H, hd / 8, reinterpret_cast<uint4*>(out), ldo / 8);
    VPF_RETURN_LAUNCH();
}

VPF_API int vpf_cls_attn_fold_bf16(const uint16_t* tokens, int64_t n_part, int N, int H, const float* planes,
                                   int64_t plane_rows, float eps, const uint16_t* G, int64_t ldg, const uint16_t* q,
                                   int64_t ldq, const float* bk, float scale, uint16_t* out, int64_t ldo,
                                   void* stream) {
    if (n_part < 0 || N <= 0 || N > NMAX || !(H == 6 || H == 12 || H == 16) || !(eps >= 0.f)) return VPF_ERR_ARG;
    const int64_t D = 64 * H;
    if (!tokens || !planes || !G || !q || !bk || !out || plane_rows < n_part * N || ldg < H * D || ldq < D ||
        ldo < H * D || (ldg & 7) || (ldo & 3) || n_part > INT32_MAX || ((uintptr_t)planes & 7) ||
        ((uintptr_t)G & 15) || ((uintptr_t)out & 7) || ((uintptr_t)tokens & 15))
        return VPF_ERR_ARG;
    if (n_part == 0) return 0;
    const float sl2 = scale * 1.44269504088896341f;
    hipStream_t s = (hipStream_t)stream;
    const bf16_t* t = reinterpret_cast<const bf16_t*>(tokens);
    const bf16_t* g = reinterpret_cast<const bf16_t*>(G);
    const bf16_t* qq = reinterpret_cast<const bf16_t*>(q);
    bf16_t* o = reinterpret_cast<bf16_t*>(out);
    if (H == 16)
        hipLaunchKernelGGL(k_cls_attn_fold<16>, dim3((unsigned)n_part), dim3(256), 0, s, t, N, planes, plane_rows,
                           eps, g, ldg, qq, ldq, bk, sl2, o, ldo);
    else if (H == 12)
        hipLaunchKernelGGL(k_cls_attn_fold<12>, dim3((unsigned)n_part), dim3(256), 0, s, t, N, planes, plane_rows,
                           eps, g, ldg, qq, ldq, bk, sl2, o, ldo);
    else
        hipLaunchKernelGGL(k_cls_attn_fold<6>, dim3((unsigned)n_part), dim3(256), 0, s, t, N, planes, plane_rows,
                           eps, g, ldg, qq, ldq, bk, sl2, o, ldo);
    VPF_RETURN_LAUNCH();
}
