// fp32 parity-mode GEMM (SURVEY.md §7 hard part (iii)): the same contract and epilogues as
// vpf_gemm_bf16, computed on gfx950's exact-f32 MFMA (v_mfma_f32_32x32x2_f32: one rounding per product,
// no reduced-precision path). Used only when the tracker runs with model.dtype = fp32 so that its
// per-frame state can be held to 1e-4 relative against the fp32 CPU oracle; performance is secondary.
//
// 128x128 tile, BK = 32, 256 threads = 4 waves (2 x 2), each wave 64x64 = 2x2 MFMA tiles. Operands are
// staged by 16-B loads into padded LDS rows (33 floats: conflict-free scalar column reads).
// Operands are swapped (W as A) so each lane holds 4 consecutive output columns of one row.
#include "vpf_common.h"
#include "../../include/vpf.h"

using namespace vpf;

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int TB = 128, KB = 32, LDR = KB + 1;

template <int EPI>
__global__ __launch_bounds__(256) void k_gemm_f32(const float* __restrict__ A, int lda, const float* __restrict__ W,
                                                  const float* __restrict__ bias, const float* residual,
                                                  const float* __restrict__ pos, int g2,
                                                  const float2* __restrict__ stats, const float* __restrict__ colsum,
                                                  float* C, int ldc, int M, int N, int K) {
    __shared__ float As[TB * LDR];
    __shared__ float Ws[TB * LDR];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int tiles_n = (N + TB - 1) / TB;
    const int tm = blockIdx.x / tiles_n, tn = blockIdx.x - (blockIdx.x / tiles_n) * tiles_n;
    const int m0 = tm * TB, n0 = tn * TB;
    const int wm = wid >> 1, wn = wid & 1;
    f32x16 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = f32x16{};
    const int l32 = lane & 31, hh = lane >> 5;
    for (int k0 = 0; k0 < K; k0 += KB) {
        // stage 128 rows x 32 floats of each operand: 1024 float4 per operand, 4 per thread
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int idx = tid + it * 256;
            const int r = idx >> 3, c4 = (idx & 7) * 4;
            const int ra = min(m0 + r, M - 1), rb = min(n0 + r, N - 1);
            const float4 av = *reinterpret_cast<const float4*>(A + (int64_t)ra * lda + k0 + c4);
            const float4 wv = *reinterpret_cast<const float4*>(W + (int64_t)rb * K + k0 + c4);
            float* ad = As + r * LDR + c4;
            float* wd = Ws + r * LDR + c4;
            ad[0] = av.x; ad[1] = av.y; ad[2] = av.z; ad[3] = av.w;
            wd[0] = wv.x; wd[1] = wv.y; wd[2] = wv.z; wd[3] = wv.w;
        }
        __syncthreads();
#pragma unroll 4
        for (int kk = 0; kk < KB; kk += 2) {
            float af[2], wf[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                af[t] = As[(wm * 64 + t * 32 + l32) * LDR + kk + hh];
                wf[t] = Ws[(wn * 64 + t * 32 + l32) * LDR + kk + hh];
            }
#pragma unroll
            for (int tnn = 0; tnn < 2; ++tnn)
#pragma unroll
                for (int tmm = 0; tmm < 2; ++tmm)
                    acc[tnn][tmm] = __builtin_amdgcn_mfma_f32_32x32x2f32(wf[tnn], af[tmm], acc[tnn][tmm], 0, 0, 0);
        }
        __syncthreads();
    }
    // epilogue: acc[tnn][tmm] holds D[n][m]: m = lane col, n = (r&3) + 8(r>>2) + 4hh
#pragma unroll
    for (int tmm = 0; tmm < 2; ++tmm) {
        const int m = m0 + wm * 64 + tmm * 32 + l32;
        if (m >= M) continue;
        constexpr bool LN = (EPI == VPF_EPI_LN || EPI == VPF_EPI_LN_GELU);
        float2 rs = make_float2(1.f, 0.f);
        if constexpr (LN) { const float2 st = stats[m]; rs = make_float2(st.y, -st.y * st.x); }
        int64_t orow = m;
        int pi = 0;
        if constexpr (EPI == VPF_EPI_PATCH) { pi = m % g2; orow = (int64_t)(m / g2) * (g2 + 1) + 1 + pi; }
#pragma unroll
        for (int tnn = 0; tnn < 2; ++tnn)
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
                const int n = n0 + wn * 64 + tnn * 32 + 8 * g4 + 4 * hh;
                if (n >= N) continue;
                const float4 bv = *reinterpret_cast<const float4*>(bias + n);
                float v[4] = {acc[tnn][tmm][4 * g4] + bv.x, acc[tnn][tmm][4 * g4 + 1] + bv.y,
                              acc[tnn][tmm][4 * g4 + 2] + bv.z, acc[tnn][tmm][4 * g4 + 3] + bv.w};
                if constexpr (LN) {
                    const float4 cv = *reinterpret_cast<const float4*>(colsum + n);
                    v[0] = fmaf(rs.x, acc[tnn][tmm][4 * g4], fmaf(rs.y, cv.x, bv.x));
                    v[1] = fmaf(rs.x, acc[tnn][tmm][4 * g4 + 1], fmaf(rs.y, cv.y, bv.y));
                    v[2] = fmaf(rs.x, acc[tnn][tmm][4 * g4 + 2], fmaf(rs.y, cv.z, bv.z));
                    v[3] = fmaf(rs.x, acc[tnn][tmm][4 * g4 + 3], fmaf(rs.y, cv.w, bv.w));
                }
                if constexpr (EPI == VPF_EPI_BIAS_GELU || EPI == VPF_EPI_LN_GELU) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = 0.5f * v[e] * (1.0f + erff(v[e] * 0.70710678118654752f));
                }
                if constexpr (EPI == VPF_EPI_BIAS_RESIDUAL) {
                    const float4 rv = *reinterpret_cast<const float4*>(residual + (int64_t)m * ldc + n);
                    v[0] += rv.x; v[1] += rv.y; v[2] += rv.z; v[3] += rv.w;
                }
                if constexpr (EPI == VPF_EPI_PATCH) {
                    const float4 pv = *reinterpret_cast<const float4*>(pos + (int64_t)(1 + pi) * N + n);
                    v[0] += pv.x; v[1] += pv.y; v[2] += pv.z; v[3] += pv.w;
                }
                *reinterpret_cast<float4*>(C + orow * ldc + n) = make_float4(v[0], v[1], v[2], v[3]);
            }
    }
}

}  // namespace

#define VPF_GEMMF_LAUNCH(E)                                                                                  \
    hipLaunchKernelGGL(k_gemm_f32<E>, grid, block, 0, s, A, (int)lda, W, bias, residual, pos, patch_rows,           \
                       reinterpret_cast<const float2*>(row_stats), colsum, C, (int)ldc, m, n, k)

VPF_API int vpf_gemm_f32(const float* A, int64_t lda, const float* W, const float* bias, const float* residual,
                         const float* pos, int patch_rows, const float* row_stats, const float* colsum, float* C,
                         int64_t ldc, int64_t M, int64_t N, int64_t K, int epilogue, void* stream) {
    if (M <= 0 || N <= 0 || K <= 0 || K % KB != 0 || N % 8 != 0 || lda < K || lda % 4 != 0 || ldc < N ||
        ldc % 4 != 0)
        return VPF_ERR_ARG;
    if (M > INT32_MAX / 2 || N > 65536 || K > 65536 || lda > INT32_MAX / 2 || ldc > INT32_MAX / 2) return VPF_ERR_ARG;
    if (!A || !W || !bias || !C) return VPF_ERR_ARG;
    if (epilogue == VPF_EPI_BIAS_RESIDUAL && !residual) return VPF_ERR_ARG;
    if (epilogue == VPF_EPI_PATCH && (!pos || patch_rows <= 0 || M % patch_rows != 0)) return VPF_ERR_ARG;
    if ((epilogue == VPF_EPI_LN || epilogue == VPF_EPI_LN_GELU) && (!row_stats || !colsum)) return VPF_ERR_ARG;
    const int64_t tiles = ((M + TB - 1) / TB) * ((N + TB - 1) / TB);
    if (tiles > INT32_MAX) return VPF_ERR_ARG;
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((unsigned)tiles), block(256);
    const int m = (int)M, n = (int)N, k = (int)K;
    switch (epilogue) {
        case VPF_EPI_BIAS: VPF_GEMMF_LAUNCH(VPF_EPI_BIAS); break;
        case VPF_EPI_BIAS_GELU: VPF_GEMMF_LAUNCH(VPF_EPI_BIAS_GELU); break;
        case VPF_EPI_BIAS_RESIDUAL: VPF_GEMMF_LAUNCH(VPF_EPI_BIAS_RESIDUAL); break;
        case VPF_EPI_PATCH: VPF_GEMMF_LAUNCH(VPF_EPI_PATCH); break;
        case VPF_EPI_LN: VPF_GEMMF_LAUNCH(VPF_EPI_LN); break;
        case VPF_EPI_LN_GELU: VPF_GEMMF_LAUNCH(VPF_EPI_LN_GELU); break;
        default: return VPF_ERR_ARG;
    }
    VPF_RETURN_LAUNCH();
}
