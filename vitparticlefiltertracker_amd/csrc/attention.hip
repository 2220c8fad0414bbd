// Multi-head self-attention per (particle, head): out = softmax(q k^T * scale) v,
// non-causal, N tokens (197 for /16@224, 577 for /14@336), head_dim 64.
//
// bf16 path (vpf_attention_bf16): one 256-thread workgroup per (particle, head). K and V of the head
// are staged once into LDS (N rounded up to 64 keys; padding rows zero):
//   K image: 128-B rows, 16-B chunk c of row r at c ^ ((r >> 1) & 7)   -> ds_read_b128 conflict-free
//   V image: 128-B rows, 16-B chunk c of row r at c ^ (((r >> 1) & 1) << 2) -> ds_read_b64_tr_b16
//            conflict-free (T10 hardware-transposed read feeds V^T as the MFMA A operand).
// Each wave takes 32-query strips. "Swapped" QK^T (K as A, Q as B) on v_mfma_f32_32x32x16_bf16 puts one
// query per lane column and its keys in the lane's 16 accumulator registers, so the online-softmax row
// max / sum is register-local plus one cross-half shuffle, and the bf16-packed probabilities are
// directly the B operand of O^T = V^T P^T (cdna_hip_programming.md §3, accumulator as next operand).
// Keys are processed in blocks of 64 with online softmax (exp2 with scale*log2e folded in), so the
// register footprint does not grow with N.
//
// fp32 parity path (vpf_attention_f32): one thread per query, K/V of the head in LDS as fp32, exact
// expf softmax (N <= 256).
#include "vpf_common.h"
#include "../../include/vpf.h"

using namespace vpf;

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int HD = 64;
constexpr int ROWB = HD * 2;  // 128 B per K/V row

__device__ __forceinline__ int k_off(int r, int c) { return r * ROWB + ((c ^ ((r >> 1) & 7)) << 4); }
__device__ __forceinline__ int v_off(int r, int c) { return r * ROWB + ((c ^ (((r >> 1) & 1) << 2)) << 4); }

__device__ __forceinline__ bf16x4 ds_read_tr(const char* lds_base, int byte_off) {
    typedef __attribute__((address_space(3))) bf16x4 lds_v4;
    const lds_v4* p = reinterpret_cast<const lds_v4*>(
        (__attribute__((address_space(3))) const char*)((size_t)lds_base) + byte_off);
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<lds_v4*>(p));
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// One key step of T 32-key tiles (T = 1 or 2) for a 32-query strip: S^T = K Q^T on MFMA, online softmax
// update of (m, l, O), O^T += V^T P^T with V^T fragments from transposed LDS reads. MASK: this step contains
// padded keys (only the last step). The O / l rescale is skipped when no query's running max moved in this
// step (wave-uniform test), which is the common case after the first key tiles.
template <int T, bool MASK>
__device__ __forceinline__ void attn_step(const char* Ks, const char* Vs, int kb, int N, int lane, const bf16x8 qf[4],
                                          float scale_log2, float& m, float& l, f32x16& o0, f32x16& o1) {
    const int l32 = lane & 31, hh = lane >> 5;
    f32x16 s[T];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        s[t] = f32x16{};
        const int kr = kb + t * 32 + l32;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + k_off(kr, ks * 2 + hh));
            s[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], s[t], 0, 0, 0);
        }
    }
    float bm = -INFINITY;
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if constexpr (MASK) {
                const int key = kb + t * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
                if (key >= N) s[t][r] = -INFINITY;
            }
            bm = fmaxf(bm, s[t][r]);
        }
    bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
    if (__builtin_expect(__any(bm > m), 0) || kb == 0) {
        const float mn = fmaxf(m, bm);
        const float alpha = __builtin_amdgcn_exp2f((m - mn) * scale_log2);
        m = mn;
        l *= alpha;
        const f32x2 a2 = {alpha, alpha};
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
            f32x2 x0 = {o0[r], o0[r + 1]}, x1 = {o1[r], o1[r + 1]};
            x0 *= a2; x1 *= a2;
            o0[r] = x0.x; o0[r + 1] = x0.y; o1[r] = x1.x; o1[r + 1] = x1.y;
        }
    }
    const float msc = m * scale_log2;
    bf16x8 pf[T][2];
#pragma unroll
    for (int t = 0; t < T; ++t) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float p = __builtin_amdgcn_exp2f(fmaf(s[t][r], scale_log2, -msc));
            s[t][r] = p;
            l += p;
        }
#pragma unroll
        for (int st = 0; st < 2; ++st) {
            const uint4 u = make_uint4(pack_bf2(s[t][8 * st + 0], s[t][8 * st + 1]), pack_bf2(s[t][8 * st + 2], s[t][8 * st + 3]),
                                       pack_bf2(s[t][8 * st + 4], s[t][8 * st + 5]), pack_bf2(s[t][8 * st + 6], s[t][8 * st + 7]));
            pf[t][st] = __builtin_bit_cast(bf16x8, u);
        }
    }
    const int grp = lane >> 4, gi = lane & 15;
    const int rq = gi >> 2, cp = gi & 3;
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int st = 0; st < 2; ++st) {
            const int rbase = kb + t * 32 + st * 16 + 4 * (grp >> 1) + rq;
#pragma unroll
            for (int dt = 0; dt < 2; ++dt) {
                const int col = dt * 32 + 16 * (grp & 1) + 4 * cp;
                const int c16 = col >> 3, inner = (col & 7) * 2;
                const bf16x4 lo = ds_read_tr(Vs, v_off(rbase, c16) + inner);
                const bf16x4 hi = ds_read_tr(Vs, v_off(rbase + 8, c16) + inner);
                const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                if (dt == 0) o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[t][st], o0, 0, 0, 0);
                else o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[t][st], o1, 0, 0, 0);
            }
        }
}

// One workgroup per (particle, head); one wave per 32-query strip (up to 8 waves, strips beyond loop).
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void k_attn_bf16(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ out,
                                                   int N, int H, float scale_log2, int q_rows) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int NP = (N + 31) & ~31;       // keys padded to whole 32-key MFMA tiles
    char* Ks = smem;
    char* Vs = smem + NP * ROWB;
    const int bh = blockIdx.x;
    const int b = bh / H, h = bh - (bh / H) * H;
    const int D = H * HD;
    const int64_t row0 = (int64_t)b * N;
    const bf16_t* qbase = qkv + row0 * 3 * D + h * HD;
    const bf16_t* kbase = qbase + D;
    const bf16_t* vbase = qbase + 2 * D;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nw = blockDim.x >> 6;

    for (int idx = tid; idx < NP * 8; idx += blockDim.x) {
        const int r = idx >> 3, c = idx & 7;
        uint4 kv = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
        if (r < N) {
            kv = *reinterpret_cast<const uint4*>(kbase + (int64_t)r * 3 * D + c * 8);
            vv = *reinterpret_cast<const uint4*>(vbase + (int64_t)r * 3 * D + c * 8);
        }
        *reinterpret_cast<uint4*>(Ks + k_off(r, c)) = kv;
        *reinterpret_cast<uint4*>(Vs + v_off(r, c)) = vv;
    }
    __syncthreads();

    const int l32 = lane & 31, hh = lane >> 5;
    const int nstrips = (q_rows + 31) >> 5;
    for (int strip = wid; strip < nstrips; strip += nw) {
        const int q = strip * 32 + l32;
        bf16x8 qf[4];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            if (q < N) qf[ks] = *reinterpret_cast<const bf16x8*>(qbase + (int64_t)q * 3 * D + ks * 16 + hh * 8);
            else qf[ks] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
        f32x16 o0 = {}, o1 = {};
        float m = -INFINITY, l = 0.f;
        // full 32-key tiles need no mask; only the tail tile (NP - N padded keys) is masked. One S tile live
        // keeps the kernel at <= 128 VGPRs = 4 waves/SIMD (two 7-wave workgroups per CU).
        const int nfull = N & ~31;
        int kb = 0;
        for (; kb < nfull; kb += 32) attn_step<1, false>(Ks, Vs, kb, N, lane, qf, scale_log2, m, l, o0, o1);
        if (kb < NP) attn_step<1, true>(Ks, Vs, kb, N, lane, qf, scale_log2, m, l, o0, o1);
        l += __shfl_xor(l, 32, 64);
        const float inv = 1.0f / l;
        if (q < q_rows) {
            bf16_t* orow = out + (row0 + q) * D + h * HD;
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
                const int d = 8 * g4 + 4 * hh;
                *reinterpret_cast<uint2*>(orow + d) =
                    make_uint2(pack_bf2(o0[4 * g4] * inv, o0[4 * g4 + 1] * inv), pack_bf2(o0[4 * g4 + 2] * inv, o0[4 * g4 + 3] * inv));
                *reinterpret_cast<uint2*>(orow + 32 + d) =
                    make_uint2(pack_bf2(o1[4 * g4] * inv, o1[4 * g4 + 1] * inv), pack_bf2(o1[4 * g4 + 2] * inv, o1[4 * g4 + 3] * inv));
            }
        }
    }
}

// ---------------- fp32 parity path ----------------
__global__ __launch_bounds__(256) void k_attn_f32(const float* __restrict__ qkv, float* __restrict__ out, int N,
                                                  int H, float scale, int q_rows) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* Ks = reinterpret_cast<float*>(smem);
    float* Vs = Ks + N * HD;
    const int bh = blockIdx.x;
    const int b = bh / H, h = bh - (bh / H) * H;
    const int D = H * HD;
    const int64_t row0 = (int64_t)b * N;
    const float* qbase = qkv + row0 * 3 * D + h * HD;
    for (int idx = threadIdx.x; idx < N * HD; idx += blockDim.x) {
        const int r = idx / HD, c = idx - (idx / HD) * HD;
        Ks[idx] = qbase[(int64_t)r * 3 * D + D + c];
        Vs[idx] = qbase[(int64_t)r * 3 * D + 2 * D + c];
    }
    __syncthreads();
    for (int q = threadIdx.x; q < q_rows; q += blockDim.x) {
        float qv[HD];
        for (int c = 0; c < HD; ++c) qv[c] = qbase[(int64_t)q * 3 * D + c];
        float mx = -INFINITY;
        for (int k = 0; k < N; ++k) {
            float s = 0.f;
            for (int c = 0; c < HD; ++c) s = fmaf(qv[c], Ks[k * HD + c], s);
            mx = fmaxf(mx, s * scale);
        }
        float acc[HD];
        for (int c = 0; c < HD; ++c) acc[c] = 0.f;
        float l = 0.f;
        for (int k = 0; k < N; ++k) {
            float s = 0.f;
            for (int c = 0; c < HD; ++c) s = fmaf(qv[c], Ks[k * HD + c], s);
            const float p = expf(s * scale - mx);
            l += p;
            for (int c = 0; c < HD; ++c) acc[c] = fmaf(p, Vs[k * HD + c], acc[c]);
        }
        float* orow = out + (row0 + q) * D + h * HD;
        for (int c = 0; c < HD; ++c) orow[c] = acc[c] / l;
    }
}

}  // namespace

VPF_API int vpf_attention_bf16(const uint16_t* qkv, uint16_t* out, int64_t B, int N, int H, int hd, float scale,
                               int q_rows, void* stream) {
    if (B < 0 || N <= 0 || N > 640 || H <= 0 || hd != HD || B * H > INT32_MAX || q_rows < 1 || q_rows > N)
        return VPF_ERR_ARG;
    if (B == 0) return 0;
    const int NP = (N + 31) & ~31;
    const size_t lds = (size_t)NP * ROWB * 2;
    const float scale_log2 = scale * 1.44269504088896341f;
    const int strips = (q_rows + 31) / 32;
    const int threads = 64 * (strips < 8 ? strips : 8);
    static bool attr_set = false;   // benign race: idempotent attribute set
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k_attn_bf16, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    hipLaunchKernelGGL(k_attn_bf16, dim3((unsigned)(B * H)), dim3(threads), lds, (hipStream_t)stream, qkv, out, N,
                       H, scale_log2, q_rows);
    VPF_RETURN_LAUNCH();
}

VPF_API int vpf_attention_f32(const float* qkv, float* out, int64_t B, int N, int H, int hd, float scale,
                              int q_rows, void* stream) {
    if (B < 0 || N <= 0 || N > 256 || H <= 0 || hd != HD || B * H > INT32_MAX || q_rows < 1 || q_rows > N)
        return VPF_ERR_ARG;
    if (B == 0) return 0;
    const size_t lds = (size_t)N * HD * 4 * 2;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k_attn_f32, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    hipLaunchKernelGGL(k_attn_f32, dim3((unsigned)(B * H)), dim3(256), lds, (hipStream_t)stream, qkv, out, N, H,
                       scale, q_rows);
    VPF_RETURN_LAUNCH();
}
