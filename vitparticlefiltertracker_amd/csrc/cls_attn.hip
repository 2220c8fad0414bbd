// Last encoder block, CLS query only, without materialising K and V (SURVEY.md §8a H6 + H9; the last block's
// outputs other than the CLS row feed nothing).
//
// With the LayerNorm folded as everywhere else (W' = W diag(gamma), b' = b + W beta, LNraw_j = (h_j - mean_j)
// rstd_j), the CLS query's attention in head h is
//   s_hj = q_h . k_hj = LNraw_j . G_h + c0_h,    G_h = W'_k,h^T q_h  (a D-vector),  c0_h = q_h . b'_k,h
//   o_h  = sum_j p_hj v_hj = W'_v,h U_h + b'_v,h,   U_h = sum_j p_hj LNraw_j,   p_h = softmax_j(s_h * scale)
// so the K / V GEMMs over all N tokens (2 x 2 N D^2 flops per particle) become one D-long dot and one D-long
// axpy per (token, head): this kernel. G comes from a block-diagonal GEMM of the CLS queries, and o from a
// block-diagonal GEMM of U (vit.py).
//
// One 256-thread workgroup per particle; wave w takes tokens w, w+4, ...; lane l owns dims [H l, H l + H) of
// every row (D = 64 H: a row is one coalesced 2D-byte wave load).
//   pass 1: row statistics from the producer's statistics planes (kept in LDS), LNraw of the lane's dims, H
//           partial dots with G (v_dot2_f32_bf16, G resident as bf16 pairs), a butterfly over the wave (all
//           lanes end with the same bits) -> scores in LDS;
//   softmax per head over the N scores (exact, two-pass, exp2 domain);
//   pass 2: U_h += p_hj LNraw_j (H x H fp32 accumulators per lane), the four waves' partial U summed in LDS,
//           out = U as bf16 [H][D] per particle.
#include "vpf_common.h"
#include "../../include/vpf.h"

using namespace vpf;

namespace {

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
constexpr int NMAX = 256;

template <int H>
__global__ __launch_bounds__(256) void k_cls_attn_fold(const bf16_t* __restrict__ tok, int N,
                                                       const float* __restrict__ planes, int64_t plane_rows,
                                                       float eps, const bf16_t* __restrict__ G, int64_t ldg,
                                                       const bf16_t* __restrict__ q, int64_t ldq,
                                                       const float* __restrict__ bk, float scale_log2,
                                                       bf16_t* __restrict__ out, int64_t ldo) {
    constexpr int D = 64 * H;
    constexpr int HP = H / 2;   // bf16 pairs per lane slice of a row
    __shared__ float sc[H][NMAX];          // scores, then probabilities
    __shared__ float2 rs[NMAX];            // (mean, rstd) per token
    __shared__ float usum[H * H * 64];     // the waves' partial U
    __shared__ float c0s[H];
    const int p = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const bf16_t* trow0 = tok + (int64_t)p * N * D;

    // c0_h = q_h . b'_k,h (wave h % 4 reduces head h)
    for (int h = wid; h < H; h += 4) {
        float a = bf2f(q[(int64_t)p * ldq + h * 64 + lane]) * bk[h * 64 + lane];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
        if (lane == 0) c0s[h] = a;
    }
    // G slice of this lane: H heads x H dims, bf16 pairs
    uint32_t g[H][HP];
#pragma unroll
    for (int h = 0; h < H; ++h) {
        const uint32_t* gp = reinterpret_cast<const uint32_t*>(G + (int64_t)p * ldg + (int64_t)h * D + H * lane);
#pragma unroll
        for (int e = 0; e < HP; ++e) g[h][e] = gp[e];
    }
    __syncthreads();

    // ---- pass 1: scores ----
    for (int j = wid; j < N; j += 4) {
        // row statistics: lane t < H (= the number of 64-column planes) fetches plane t, 16-lane butterfly
        float2 st = make_float2(0.f, 0.f);
        if (lane < H) st = *reinterpret_cast<const float2*>(planes + ((int64_t)lane * plane_rows + (int64_t)p * N + j) * 2);
        float s1 = st.x, s2 = st.y;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            s1 += __shfl_xor(s1, o, 64);
            s2 += __shfl_xor(s2, o, 64);
        }
        s1 = __shfl(s1, 0, 64);
        s2 = __shfl(s2, 0, 64);
        const float mean = s1 * (1.0f / D);
        const float rstd = __builtin_amdgcn_rsqf(fmaxf(s2 * (1.0f / D) - mean * mean, 0.f) + eps);
        if (lane == 0) rs[j] = make_float2(mean, rstd);
        const uint32_t* rp = reinterpret_cast<const uint32_t*>(trow0 + (int64_t)j * D + H * lane);
        uint32_t xb[HP];
#pragma unroll
        for (int e = 0; e < HP; ++e) {
            const uint32_t w = rp[e];
            xb[e] = pack_bf2((bf2f((bf16_t)(w & 0xffff)) - mean) * rstd, (bf2f((bf16_t)(w >> 16)) - mean) * rstd);
        }
        float s[H];
#pragma unroll
        for (int h = 0; h < H; ++h) {
            float a = 0.f;
#pragma unroll
            for (int e = 0; e < HP; ++e)
                a = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, xb[e]),
                                                   __builtin_bit_cast(bf16x2_t, g[h][e]), a, false);
            s[h] = a;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
#pragma unroll
            for (int h = 0; h < H; ++h) s[h] += __shfl_xor(s[h], o, 64);
        if (lane < H) {
            float v = s[0];
#pragma unroll
            for (int h = 1; h < H; ++h) v = lane == h ? s[h] : v;
            sc[lane][j] = v;
        }
    }
    __syncthreads();

    // ---- softmax per head (exp2 domain, scale folded) ----
    for (int h = wid; h < H; h += 4) {
        const float c0 = c0s[h];
        float mx = -INFINITY;
        for (int j = lane; j < N; j += 64) mx = fmaxf(mx, (sc[h][j] + c0) * scale_log2);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
        float sum = 0.f;
        for (int j = lane; j < N; j += 64) {
            const float e = __builtin_amdgcn_exp2f((sc[h][j] + c0) * scale_log2 - mx);
            sc[h][j] = e;
            sum += e;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
        const float inv = 1.0f / sum;
        for (int j = lane; j < N; j += 64) sc[h][j] *= inv;
    }
    __syncthreads();

    // ---- pass 2: U_h = sum_j p_hj LNraw_j ----
    float u[H][H];
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
        for (int i = 0; i < H; ++i) u[h][i] = 0.f;
    for (int j = wid; j < N; j += 4) {
        const float2 mr = rs[j];
        const uint32_t* rp = reinterpret_cast<const uint32_t*>(trow0 + (int64_t)j * D + H * lane);
        float x[H];
#pragma unroll
        for (int e = 0; e < HP; ++e) {
            const uint32_t w = rp[e];
            x[2 * e] = (bf2f((bf16_t)(w & 0xffff)) - mr.x) * mr.y;
            x[2 * e + 1] = (bf2f((bf16_t)(w >> 16)) - mr.x) * mr.y;
        }
#pragma unroll
        for (int h = 0; h < H; ++h) {
            const float pr = sc[h][j];
#pragma unroll
            for (int i = 0; i < H; ++i) u[h][i] = fmaf(pr, x[i], u[h][i]);
        }
    }
    for (int w = 0; w < 4; ++w) {   // sum the waves' partial U (fixed order)
        if (wid == w) {
#pragma unroll
            for (int h = 0; h < H; ++h)
#pragma unroll
                for (int i = 0; i < H; ++i) {
                    float* up = &usum[(h * H + i) * 64 + lane];
                    *up = w == 0 ? u[h][i] : *up + u[h][i];
                }
        }
        __syncthreads();
    }
    // out[h][H lane + i], as bf16 pairs; wave w writes heads w, w+4, ...
    for (int h = wid; h < H; h += 4) {
        uint32_t* op = reinterpret_cast<uint32_t*>(out + (int64_t)p * ldo + (int64_t)h * D + H * lane);
#pragma unroll
        for (int e = 0; e < HP; ++e)
            op[e] = pack_bf2(usum[(h * H + 2 * e) * 64 + lane], usum[(h * H + 2 * e + 1) * 64 + lane]);
    }
}

}  // namespace

VPF_API int vpf_cls_attn_fold_bf16(const uint16_t* tokens, int64_t n_part, int N, int H, const float* planes,
                                   int64_t plane_rows, float eps, const uint16_t* G, int64_t ldg, const uint16_t* q,
                                   int64_t ldq, const float* bk, float scale, uint16_t* out, int64_t ldo,
                                   void* stream) {
    if (n_part < 0 || N <= 0 || N > NMAX || !(H == 6 || H == 12) || !(eps >= 0.f)) return VPF_ERR_ARG;
    const int64_t D = 64 * H;
    if (!tokens || !planes || !G || !q || !bk || !out || plane_rows < n_part * N || ldg < H * D || ldq < D ||
        ldo < H * D || (ldg & 1) || (ldo & 1) || n_part > INT32_MAX || ((uintptr_t)planes & 7) ||
        ((uintptr_t)G & 3) || ((uintptr_t)out & 3) || ((uintptr_t)tokens & 3))
        return VPF_ERR_ARG;
    if (n_part == 0) return 0;
    const float sl2 = scale * 1.44269504088896341f;
    hipStream_t s = (hipStream_t)stream;
    const bf16_t* t = reinterpret_cast<const bf16_t*>(tokens);
    const bf16_t* g = reinterpret_cast<const bf16_t*>(G);
    const bf16_t* qq = reinterpret_cast<const bf16_t*>(q);
    bf16_t* o = reinterpret_cast<bf16_t*>(out);
    if (H == 12)
        hipLaunchKernelGGL(k_cls_attn_fold<12>, dim3((unsigned)n_part), dim3(256), 0, s, t, N, planes, plane_rows,
                           eps, g, ldg, qq, ldq, bk, sl2, o, ldo);
    else
        hipLaunchKernelGGL(k_cls_attn_fold<6>, dim3((unsigned)n_part), dim3(256), 0, s, t, N, planes, plane_rows,
                           eps, g, ldg, qq, ldq, bk, sl2, o, ldo);
    VPF_RETURN_LAUNCH();
}
