// LayerNorm rows and the fused final-LN -> cosine -> fixed-point weight kernel
// (H9 + H10, SPEC S4/S5).
//
// One wave per row (HBM-bound: 2 bytes in + 2 bytes out per element for bf16). Lane i holds the 4-element
// chunks i, i+64, i+128, i+192 (D <= 1024, D % 4 == 0) in registers, so the row is read once; mean and
// variance are two wave reductions over the register copy (two-pass, fp32).
#include "vpf_common.h"
#include "../../include/vpf.h"

using namespace vpf;

namespace {

template <typename T> struct Vec4;
template <> struct Vec4<float> {
    static __device__ __forceinline__ void load(const float* p, float v[4]) {
        const float4 x = *reinterpret_cast<const float4*>(p);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    }
    static __device__ __forceinline__ void store(float* p, const float v[4]) {
        *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    }
};
template <> struct Vec4<bf16_t> {
    static __device__ __forceinline__ void load(const bf16_t* p, float v[4]) {
        const uint2 x = *reinterpret_cast<const uint2*>(p);
        v[0] = bf2f((bf16_t)(x.x & 0xffff)); v[1] = bf2f((bf16_t)(x.x >> 16));
        v[2] = bf2f((bf16_t)(x.y & 0xffff)); v[3] = bf2f((bf16_t)(x.y >> 16));
    }
    static __device__ __forceinline__ void store(bf16_t* p, const float v[4]) {
        *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
    }
};

// Normalise one row held as up to 4 chunks of 4 per lane. Returns values in v (in place).
template <typename T>
__device__ __forceinline__ void ln_row(const T* __restrict__ x, int D, const float* __restrict__ g,
                                       const float* __restrict__ b, float eps, int lane, float v[16]) {
    const int nch = D >> 2;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int c = lane + 64 * i;
        if (c < nch) {
            Vec4<T>::load(x + 4 * c, v + 4 * i);
            s += (v[4 * i] + v[4 * i + 1]) + (v[4 * i + 2] + v[4 * i + 3]);
        } else {
            v[4 * i] = v[4 * i + 1] = v[4 * i + 2] = v[4 * i + 3] = 0.f;
        }
    }
    const float mean = wave_sum(s) / (float)D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int c = lane + 64 * i;
        if (c < nch) {
#pragma unroll
            for (int e = 0; e < 4; ++e) { const float d = v[4 * i + e] - mean; q = fmaf(d, d, q); }
        }
    }
    const float var = wave_sum(q) / (float)D;
    const float rstd = 1.0f / sqrtf(var + eps);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int c = lane + 64 * i;
        if (c < nch) {
            const float4 gg = *reinterpret_cast<const float4*>(g + 4 * c);
            const float4 bb = *reinterpret_cast<const float4*>(b + 4 * c);
            v[4 * i + 0] = (v[4 * i + 0] - mean) * rstd * gg.x + bb.x;
            v[4 * i + 1] = (v[4 * i + 1] - mean) * rstd * gg.y + bb.y;
            v[4 * i + 2] = (v[4 * i + 2] - mean) * rstd * gg.z + bb.z;
            v[4 * i + 3] = (v[4 * i + 3] - mean) * rstd * gg.w + bb.w;
        }
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_layernorm(const T* __restrict__ x, int64_t rows, int D, int64_t xs,
                                                   const float* __restrict__ g, const float* __restrict__ b,
                                                   float eps, T* __restrict__ y, int64_t ys) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    float v[16];
    ln_row<T>(x + row * xs, D, g, b, eps, lane, v);
    const int nch = D >> 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int c = lane + 64 * i;
        if (c < nch) Vec4<T>::store(y + row * ys + 4 * c, v + 4 * i);
    }
}

template <typename T, bool DO_LN>
__global__ __launch_bounds__(256) void k_cls_weight(const T* __restrict__ tok, int64_t n, int N, int D,
                                                    const float* __restrict__ g, const float* __restrict__ b,
                                                    float eps, const float* __restrict__ tmpl, float lam,
                                                    double scale, float* __restrict__ feat,
                                                    float* __restrict__ sim_out, int64_t* __restrict__ Q) {
    const int lane = threadIdx.x & 63;
    const int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p >= n) return;
    float v[16];
    const int nch = D >> 2;
    if constexpr (DO_LN) {
        ln_row<T>(tok + p * (int64_t)N * D, D, g, b, eps, lane, v);
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int c = lane + 64 * i;
            if (c < nch) Vec4<T>::load(tok + p * (int64_t)N * D + 4 * c, v + 4 * i);
        }
    }
    float dot = 0.f, nn = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int c = lane + 64 * i;
        if (c < nch) {
            const float4 t = *reinterpret_cast<const float4*>(tmpl + 4 * c);
            dot = fmaf(v[4 * i], t.x, dot); dot = fmaf(v[4 * i + 1], t.y, dot);
            dot = fmaf(v[4 * i + 2], t.z, dot); dot = fmaf(v[4 * i + 3], t.w, dot);
            nn = fmaf(v[4 * i], v[4 * i], nn); nn = fmaf(v[4 * i + 1], v[4 * i + 1], nn);
            nn = fmaf(v[4 * i + 2], v[4 * i + 2], nn); nn = fmaf(v[4 * i + 3], v[4 * i + 3], nn);
            if (feat) *reinterpret_cast<float4*>(feat + p * D + 4 * c) =
                make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
        }
    }
    dot = wave_sum(dot);
    nn = wave_sum(nn);
    if (lane == 0) {
        // SPEC S5: a cosine is <= 1 in exact arithmetic; clamping the fp32 value there keeps w <= 1 and so
        // Q_i <= 2^K (the K + ceil(log2 P) <= 62 budget). A zero row has sim 0; a row with a NaN / inf (or
        // whose squared norm overflows fp32) has sim NaN and zero weight.
        const bool finite = isfinite(dot) && isfinite(nn);
        const float sim = !finite ? __builtin_nanf("") : (nn > 0.f ? dot / sqrtf(nn) : 0.f);
        const float w = finite ? fixed_expf(lam * (fminf(sim, 1.0f) - 1.0f)) : 0.0f;
        Q[p] = (int64_t)floor((double)w * scale);
        if (sim_out) sim_out[p] = sim;
    }
}

// Row statistics for the LayerNorm folded into the next GEMM (vpf_gemm_bf16 EPI_LN*): out[r] = {mean, rstd}.
// Half a wave (32 lanes) per row, 16-B loads, two-pass variance on the register copy; grid-stride.
template <typename T>
__global__ __launch_bounds__(256) void k_row_stats(const T* __restrict__ x, int64_t rows, int D, int64_t xs,
                                                   float eps, float2* __restrict__ out) {
    constexpr int EPC = 16 / sizeof(T);               // elements per 16-B chunk
    constexpr int MAXC = 1024 / EPC / 32;             // chunks per lane for D <= 1024
    const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
    const int nch = D / EPC;
    // wave-uniform loop over row pairs: lanes 0-31 take row 2p, lanes 32-63 row 2p+1
    for (int64_t pr = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); 2 * pr < rows; pr += (int64_t)gridDim.x * 4) {
        const int64_t row = 2 * pr + half;
        const bool valid = row < rows;
        float v[MAXC][EPC];
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < MAXC; ++i) {
            const int c = l32 + 32 * i;
            if (valid && c < nch) {
                const uint4 u = *reinterpret_cast<const uint4*>(x + row * xs + c * EPC);
                if constexpr (sizeof(T) == 2) {
                    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        v[i][2 * e] = bf2f((bf16_t)(w[e] & 0xffff));
                        v[i][2 * e + 1] = bf2f((bf16_t)(w[e] >> 16));
                    }
                } else {
                    v[i][0] = __uint_as_float(u.x); v[i][1] = __uint_as_float(u.y);
                    v[i][2] = __uint_as_float(u.z); v[i][3] = __uint_as_float(u.w);
                }
#pragma unroll
                for (int e = 0; e < EPC; ++e) s += v[i][e];
            } else {
#pragma unroll
                for (int e = 0; e < EPC; ++e) v[i][e] = 0.f;
            }
        }
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        const float mean = s / (float)D;
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < MAXC; ++i) {
            const int c = l32 + 32 * i;
            if (c < nch) {
#pragma unroll
                for (int e = 0; e < EPC; ++e) { const float d = v[i][e] - mean; q = fmaf(d, d, q); }
            }
        }
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
        if (valid && l32 == 0) out[row] = make_float2(mean, 1.0f / sqrtf(q / (float)D + eps));
    }
}

template <typename T>
int stats_launch(const T* x, int64_t rows, int D, int64_t x_stride, float eps, float* out, void* stream) {
    constexpr int EPC = 16 / sizeof(T);
    if (rows < 0 || D <= 0 || D % EPC != 0 || D > 1024 || x_stride < D || x_stride % EPC != 0 || !out)
        return VPF_ERR_ARG;
    if (rows == 0) return 0;
    const int64_t want = (rows + 7) / 8;
    const unsigned blocks = (unsigned)(want < 8192 ? want : 8192);
    hipLaunchKernelGGL(k_row_stats<T>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, rows, D, x_stride, eps,
                       reinterpret_cast<float2*>(out));
    VPF_RETURN_LAUNCH();
}

template <typename T>
int ln_launch(const T* x, int64_t rows, int D, int64_t x_stride, const float* gamma, const float* beta,
              float eps, T* y, int64_t y_stride, void* stream) {
    if (rows < 0 || D <= 0 || D % 4 != 0 || D > 1024 || x_stride < D || y_stride < D) return VPF_ERR_ARG;
    if (rows == 0) return 0;
    const unsigned blocks = (unsigned)((rows + 3) / 4);
    hipLaunchKernelGGL(k_layernorm<T>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, rows, D, x_stride,
                       gamma, beta, eps, y, y_stride);
    VPF_RETURN_LAUNCH();
}

template <typename T>
int clsw_launch(const T* tokens, int64_t n, int N, int D, const float* gamma, const float* beta, float eps,
                const float* tmpl, float lam, int bits, float* feat_out, float* sim_out, int64_t* Q,
                void* stream) {
    if (n < 0 || N <= 0 || D <= 0 || D % 4 != 0 || D > 1024 || bits < 0 || bits > 62 || !Q || !tmpl ||
        !(lam >= 0.f) || !(lam <= 3.0e38f))
        return VPF_ERR_ARG;
    if (n == 0) return 0;
    const unsigned blocks = (unsigned)((n + 3) / 4);
    if (gamma)
        hipLaunchKernelGGL((k_cls_weight<T, true>), dim3(blocks), dim3(256), 0, (hipStream_t)stream, tokens, n, N, D,
                           gamma, beta, eps, tmpl, lam, ldexp(1.0, bits), feat_out, sim_out, Q);
    else
        hipLaunchKernelGGL((k_cls_weight<T, false>), dim3(blocks), dim3(256), 0, (hipStream_t)stream, tokens, n, N,
                           D, gamma, beta, eps, tmpl, lam, ldexp(1.0, bits), feat_out, sim_out, Q);
    VPF_RETURN_LAUNCH();
}

// H4 for LN-folded consumers with more statistics planes than their LDS holds next to the ping-pong ring (ViT-L: 16):
// the producer GEMMs' {sum, sumsq} planes combined into {mean, rstd} per row, one thread per row, with the same
// operations in the same order as the consuming GEMM's in-kernel combine (gemm_bf16.hip), so the consumer's output is
// bit-identical either way. Reads 8 B per plane and row (coalesced across the threads of a plane).
// PARTS > 0: the plane count of the encoders (3 / 12 / 16) as a constant, so all of a row's plane loads are in flight
// at once; the sums still run in plane order (the bits of the GEMMs' in-kernel combine). 0: any count.
template <int PARTS>
__global__ __launch_bounds__(256) void k_stats_combine(const float2* __restrict__ planes, int parts, int64_t pstride,
                                                       int64_t rows, float inv_k, float eps, float2* __restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    float sm = 0.f, sq = 0.f;
    if constexpr (PARTS > 0) {
        float2 st[PARTS];
#pragma unroll
        for (int p = 0; p < PARTS; ++p) st[p] = planes[p * pstride + r];
#pragma unroll
        for (int p = 0; p < PARTS; ++p) {
            sm += st[p].x;
            sq += st[p].y;
        }
    } else {
        for (int p = 0; p < parts; ++p) {
            const float2 st = planes[p * pstride + r];
            sm += st.x;
            sq += st.y;
        }
    }
    const float mean = sm * inv_k;
    const float var = fmaxf(fmaf(sq, inv_k, -mean * mean), 0.f);
    out[r] = make_float2(mean, __builtin_amdgcn_rsqf(var + eps));
}

}  // namespace

VPF_API int vpf_layernorm_bf16(const uint16_t* x, int64_t rows, int D, int64_t x_stride, const float* gamma,
                               const float* beta, float eps, uint16_t* y, int64_t y_stride, void* stream) {
    return ln_launch<bf16_t>(x, rows, D, x_stride, gamma, beta, eps, y, y_stride, stream);
}
VPF_API int vpf_layernorm_f32(const float* x, int64_t rows, int D, int64_t x_stride, const float* gamma,
                              const float* beta, float eps, float* y, int64_t y_stride, void* stream) {
    return ln_launch<float>(x, rows, D, x_stride, gamma, beta, eps, y, y_stride, stream);
}
VPF_API int vpf_row_stats_bf16(const uint16_t* x, int64_t rows, int D, int64_t x_stride, float eps, float* out,
                               void* stream) {
    return stats_launch<bf16_t>(x, rows, D, x_stride, eps, out, stream);
}
VPF_API int vpf_row_stats_f32(const float* x, int64_t rows, int D, int64_t x_stride, float eps, float* out,
                              void* stream) {
    return stats_launch<float>(x, rows, D, x_stride, eps, out, stream);
}
VPF_API int vpf_stats_combine(const float* planes, int parts, int64_t plane_stride, int64_t rows, int D, float eps,
                              float* out, void* stream) {
    if (!planes || !out || parts < 1 || parts > 64 || rows < 1 || plane_stride < rows || D < 1 || !(eps >= 0.f) ||
        ((uintptr_t)planes & 7) || ((uintptr_t)out & 7) || (rows + 255) / 256 > INT32_MAX)
        return VPF_ERR_ARG;
    const dim3 grid((unsigned)((rows + 255) / 256)), block(256);
    const float2* pl = reinterpret_cast<const float2*>(planes);
    float2* o = reinterpret_cast<float2*>(out);
    hipStream_t s = (hipStream_t)stream;
    const float inv_k = 1.0f / (float)D;
#define VPF_COMBINE(P) hipLaunchKernelGGL(k_stats_combine<P>, grid, block, 0, s, pl, parts, plane_stride, rows, inv_k, eps, o)
    switch (parts) {
        case 3: VPF_COMBINE(3); break;
        case 12: VPF_COMBINE(12); break;
        case 16: VPF_COMBINE(16); break;
        default: VPF_COMBINE(0); break;
    }
#undef VPF_COMBINE
    VPF_RETURN_LAUNCH();
}
VPF_API int vpf_cls_weight_bf16(const uint16_t* tokens, int64_t n, int N, int D, const float* gamma,
                                const float* beta, float eps, const float* tmpl, float lam, int bits,
                                float* feat_out, float* sim_out, int64_t* Q, void* stream) {
    return clsw_launch<bf16_t>(tokens, n, N, D, gamma, beta, eps, tmpl, lam, bits, feat_out, sim_out, Q, stream);
}
VPF_API int vpf_cosine_weight_f32(const float* feat, int64_t n, int D, const float* tmpl, float lam, int bits,
                                  float* sim_out, int64_t* Q, void* stream) {
    return clsw_launch<float>(feat, n, 1, D, nullptr, nullptr, 0.f, tmpl, lam, bits, nullptr, sim_out, Q, stream);
}
VPF_API int vpf_cls_weight_f32(const float* tokens, int64_t n, int N, int D, const float* gamma,
                               const float* beta, float eps, const float* tmpl, float lam, int bits,
                               float* feat_out, float* sim_out, int64_t* Q, void* stream) {
    return clsw_launch<float>(tokens, n, N, D, gamma, beta, eps, tmpl, lam, bits, feat_out, sim_out, Q, stream);
}
