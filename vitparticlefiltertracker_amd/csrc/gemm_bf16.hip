// bf16 GEMM with fused epilogues for the ViT encoder.
//
//   C[M][N] = epi( A[M][K] . W[N][K]^T ),  bf16 operands, fp32 accumulation on MFMA.
//
// Design (gfx950; MI355X_MICROARCH.md / cdna_hip_programming.md §5):
//  * 256x256 output tile, BK = 64, 512 threads = 8 waves laid out 2 (M) x 4 (N); each wave owns a
//    128 (M) x 64 (N) sub-tile = 8 x 4 fragments of v_mfma_f32_16x16x32_bf16 (128 accumulator VGPRs).
//  * Operands are staged HBM/L2 -> LDS by global_load_lds_dwordx4 (LDS-DMA, 1 KiB per wave-instruction,
//    no VGPR round trip) into a 2-stage LDS ring (2 x 64 KiB). The LDS image is lane-linear; bank
//    conflicts of the fragment reads (ds_read_b128) are removed by XOR-swizzling the per-lane SOURCE
//    address: 16-B chunk c of row r lives at physical chunk c ^ ((r >> 1) & 7) (tools/lds_banks.py:
//    conflict-free for every 16-lane group).
//  * One barrier per K-step: the DMA for K-tile t+1 is issued right after the barrier and flies while
//    the 64 MFMAs per wave of tile t run.
//  * MFMA operands are "swapped" (W fragment as A, activation fragment as B) so the accumulator holds
//    D[n][m]: each lane owns 4 consecutive output columns of one row. Epilogue: bias (+ exact-erf GELU)
//    in fp32 on the accumulators, bf16 pack, 8-B writes into a per-wave XOR-swizzled LDS image, then
//    fully coalesced 16-B row stores (+ 16-B residual reads / position-embedding adds).
//  * Workgroup -> tile mapping is XCD-aware (bijective remap, cdna_hip_programming.md §5 T1): the blocks
//    that share an XCD walk consecutive tiles of one 256-row A panel, so the panel is an L2 hit.
#include <stdlib.h>
#include "vpf_common.h"
#include "../../include/vpf.h"

using namespace vpf;

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NTHREADS = 512;
constexpr int OPERAND_BYTES = BM * BK * 2;      // 32 KiB per operand tile
constexpr int STAGE_BYTES = 2 * OPERAND_BYTES;  // A + B
constexpr int LDS_BYTES = 2 * STAGE_BYTES;      // 128 KiB
constexpr int AUX_BYTES = 4096;                 // epilogue operands: bias | colsum | row stats (1+1+2 KiB)

typedef const __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

typedef float f32x2 __attribute__((ext_vector_type(2)));

// Exact-erf GELU on packed FP32 (v_pk_fma_f32), two values at a time: x * Phi(x) with
// Phi(x) = x < 0 ? h : 1 - h,  h = erfc(|x|/sqrt2) / 2 = 1 / (2^(1/16) (1 + a1 z + ... + a6 z^6))^16,  z = |x|/sqrt2
// (Abramowitz & Stegun 7.1.28, |erf error| <= 3e-7; the 2^(1/16) and 1/sqrt2 powers are folded into the
// coefficients). One v_rcp_f32 per value and no exp; the negative tail is computed directly (no 1 - x
// cancellation). Max |GELU error| 8.7e-7 over [-12, 12] (numpy check vs scipy erf, fp32 evaluation):
// far below bf16 output resolution.
__device__ __forceinline__ f32x2 gelu_erf2(f32x2 x) {
    constexpr float c = 1.0442737824274138f;   // 2^(1/16)
    constexpr float s = 0.70710678118654752f;
    const f32x2 z = __builtin_elementwise_abs(x);
    f32x2 p = z * (0.0000430638f * c * s * s * s * s * s * s) + (0.0002765672f * c * s * s * s * s * s);
    p = p * z + (0.0001520143f * c * s * s * s * s);
    p = p * z + (0.0092705272f * c * s * s * s);
    p = p * z + (0.0422820123f * c * s * s);
    p = p * z + (0.0705230784f * c * s);
    p = p * z + c;
    p = p * p;
    p = p * p;
    p = p * p;
    p = p * p;
    const f32x2 h = {__builtin_amdgcn_rcpf(p.x), __builtin_amdgcn_rcpf(p.y)};
    const f32x2 q = 0.5f - h;
    const f32x2 sq = {__builtin_copysignf(q.x, x.x), __builtin_copysignf(q.y, x.y)};
    return x * (sq + 0.5f);
}

template <int EPI>
__global__ __launch_bounds__(NTHREADS) void k_gemm_bf16(const bf16_t* __restrict__ A, int lda,
                                                        const bf16_t* __restrict__ W,
                                                        const float* __restrict__ bias,
                                                        const bf16_t* residual,
                                                        const float* __restrict__ pos, int g2,
                                                        const float2* __restrict__ stats,
                                                        const float* __restrict__ colsum,
                                                        bf16_t* C, int ldc, int M, int N, int K, int group) {
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES + AUX_BYTES];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);

    // ---- XCD-aware bijective block -> tile remap ----
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    const int lid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    // Grouped order inside each XCD's contiguous lid range: groups of `group` A row-panels; within a group
    // the A panel index runs fastest, so the ~32 tiles an XCD has in flight cover ~group A panels x
    // 32/group W panels and both stay in that XCD's L2 (tm-major order re-fetched a 393 KB W panel per
    // tile on FC1: FETCH_SIZE 14.8 GB/launch, profiles/r1_notes.md). group = 0: plain tm-major.
    const int tiles_n = (N + BN - 1) / BN;
    int tm, tn;
    if (group > 0) {
        const int tiles_m = (M + BM - 1) / BM;
        const int per_group = group * tiles_n;
        const int g = lid / per_group, idx = lid - g * per_group;
        const int gm0 = g * group;
        const int gsz = min(group, tiles_m - gm0);
        tn = idx / gsz;
        tm = gm0 + (idx - tn * gsz);
    } else {
        tm = lid / tiles_n;
        tn = lid - tm * tiles_n;
    }
    const int m0 = tm * BM, n0 = tn * BN;

    // ---- per-lane DMA source offsets (bytes, relative to the block's panel base) ----
    const char* Ablk = reinterpret_cast<const char*>(A) + (size_t)m0 * lda * 2;
    const char* Bblk = reinterpret_cast<const char*>(W) + (size_t)n0 * K * 2;
    uint32_t offA[4], offB[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int g = i * 8 + wid;                 // wave-instruction index: rows [8g, 8g+8)
        const int row = 8 * g + (lane >> 3);
        const int pch = lane & 7;
        const int lch = pch ^ ((row >> 1) & 7);    // logical chunk stored at this physical slot
        const int ra = min(row, M - 1 - m0);
        const int rb = min(row, N - 1 - n0);
        offA[i] = (uint32_t)ra * (uint32_t)(lda * 2) + (uint32_t)(lch * 16);
        offB[i] = (uint32_t)rb * (uint32_t)(K * 2) + (uint32_t)(lch * 16);
    }
    auto stage = [&](int buf, int kt) {
        char* la = smem + buf * STAGE_BYTES;
        char* lb = la + OPERAND_BYTES;
        const uint32_t koff = (uint32_t)kt * (BK * 2);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int g = i * 8 + wid;
            __builtin_amdgcn_global_load_lds((gptr_t)(Ablk + offA[i] + koff), (lptr_t)(la + g * 1024), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((gptr_t)(Bblk + offB[i] + koff), (lptr_t)(lb + g * 1024), 16, 0, 0);
        }
    };

    const int wm = wid >> 2, wn = wid & 3;
    f32x4 acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

    // fragment read addresses (byte offsets inside an operand tile), excluding the ks chunk term
    const int fr = lane & 15, fq = lane >> 4;

    // Epilogue operands ride the first DMA wave into the aux region of LDS (bias | colsum | per-row
    // (mean, rstd)), so their latency hides under the K loop and nothing epilogue-related stays live in
    // VGPRs across it (holding them in registers cost ~10 % on the LayerNorm-folded GEMMs: 250 VGPRs).
    // Out-of-range columns / rows read clamped (valid) addresses; their values are never stored.
    constexpr bool LN = (EPI == VPF_EPI_LN || EPI == VPF_EPI_LN_GELU);
    char* aux = smem + LDS_BYTES;
    if (wid == 0)
        __builtin_amdgcn_global_load_lds((gptr_t)(bias + min(n0 + lane * 4, N - 4)), (lptr_t)aux, 16, 0, 0);
    if constexpr (LN) {
        if (wid == 1)
            __builtin_amdgcn_global_load_lds((gptr_t)(colsum + min(n0 + lane * 4, N - 4)), (lptr_t)(aux + 1024), 16, 0,
                                             0);
        const float* sd = reinterpret_cast<const float*>(stats);
        __builtin_amdgcn_global_load_lds((gptr_t)(sd + min(2 * m0 + wid * 64 + lane, 2 * M - 1)),
                                         (lptr_t)(aux + 2048 + wid * 256), 4, 0, 0);
    }
    const int nk = K / BK;
    stage(0, 0);
    for (int kt = 0; kt < nk; ++kt) {
        __syncthreads();   // vmcnt(0) + barrier: tile kt landed for every wave; tile kt-1 fully read
        if (kt + 1 < nk) stage((kt + 1) & 1, kt + 1);
        const char* la = smem + (kt & 1) * STAGE_BYTES;
        const char* lb = la + OPERAND_BYTES;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8 a[8], b[4];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int row = wm * 128 + i * 16 + fr;
                const int ch = (ks * 4 + fq) ^ ((row >> 1) & 7);
                a[i] = *reinterpret_cast<const bf16x8*>(la + row * 128 + ch * 16);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int row = wn * 64 + j * 16 + fr;
                const int ch = (ks * 4 + fq) ^ ((row >> 1) & 7);
                b[j] = *reinterpret_cast<const bf16x8*>(lb + row * 128 + ch * 16);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[j][i], 0, 0, 0);
        }
    }

    // ---------------- epilogue ----------------
    __syncthreads();   // every wave is done with the operand ring; reuse it as 8 x 16 KiB images
    char* img = smem + wid * 16384;
    float4 bv[4], cv[4];
    f32x2 rsx[8], rsy[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = (wn * 64 + j * 16 + fq * 4) * 4;
        bv[j] = *reinterpret_cast<const float4*>(aux + c);
        if constexpr (LN) cv[j] = *reinterpret_cast<const float4*>(aux + 1024 + c);
    }
    if constexpr (LN) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float2 st = *reinterpret_cast<const float2*>(aux + 2048 + (wm * 128 + i * 16 + fr) * 8);
            rsx[i] = f32x2{st.y, st.y};                       // rstd
            rsy[i] = f32x2{-st.y * st.x, -st.y * st.x};       // -rstd * mean
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            f32x2 v01, v23;
            const f32x2 a01 = {acc[j][i][0], acc[j][i][1]}, a23 = {acc[j][i][2], acc[j][i][3]};
            const f32x2 b01 = {bv[j].x, bv[j].y}, b23 = {bv[j].z, bv[j].w};
            if constexpr (LN) {
                // LN(x) W^T + b = rstd (x W'^T) - rstd mean colsum(W') + b'   (gamma folded into W', beta into b')
                const f32x2 c01 = {cv[j].x, cv[j].y}, c23 = {cv[j].z, cv[j].w};
                v01 = __builtin_elementwise_fma(rsx[i], a01, __builtin_elementwise_fma(rsy[i], c01, b01));
                v23 = __builtin_elementwise_fma(rsx[i], a23, __builtin_elementwise_fma(rsy[i], c23, b23));
            } else {
                v01 = a01 + b01;
                v23 = a23 + b23;
            }
            if constexpr (EPI == VPF_EPI_BIAS_GELU || EPI == VPF_EPI_LN_GELU) {
                v01 = gelu_erf2(v01);
                v23 = gelu_erf2(v23);
            }
            const float v0 = v01.x, v1 = v01.y, v2 = v23.x, v3 = v23.y;
            const int row = i * 16 + fr;              // row within the wave's 128-row image
            const int c8 = (j * 4 + fq) ^ (row & 15);  // swizzled 8-B chunk
            *reinterpret_cast<uint2*>(img + row * 128 + c8 * 8) = make_uint2(pack_bf2(v0, v1), pack_bf2(v2, v3));
        }
    }
    const int c16 = lane & 7;
    uint4 res[16];
    if constexpr (EPI == VPF_EPI_BIAS_RESIDUAL) {
        // all 16 residual rows of this lane in flight at once, under the LDS round trip below
#pragma unroll
        for (int it = 0; it < 16; ++it) {
            const int m = m0 + wm * 128 + it * 8 + (lane >> 3);
            const int n = n0 + wn * 64 + c16 * 8;
            res[it] = (m < M && n < N) ? *reinterpret_cast<const uint4*>(residual + (int64_t)m * ldc + n)
                                       : make_uint4(0, 0, 0, 0);
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int row = it * 8 + (lane >> 3);
        uint4 v = *reinterpret_cast<const uint4*>(img + row * 128 + ((c16 ^ ((row & 15) >> 1)) * 16));
        if (row & 1) { const uint32_t t0 = v.x, t1 = v.y; v.x = v.z; v.y = v.w; v.z = t0; v.w = t1; }
        const int m = m0 + wm * 128 + row;
        const int n = n0 + wn * 64 + c16 * 8;
        if (m >= M || n >= N) continue;
        int64_t orow = m;
        if constexpr (EPI == VPF_EPI_PATCH) {
            const int pi = m % g2;
            orow = (int64_t)(m / g2) * (g2 + 1) + 1 + pi;
            const float* pr = pos + (int64_t)(1 + pi) * N + n;
            const float4 p0 = *reinterpret_cast<const float4*>(pr);
            const float4 p1 = *reinterpret_cast<const float4*>(pr + 4);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
            const float pv[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
            uint32_t o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e)
                o[e] = pack_bf2(bf2f((bf16_t)(w[e] & 0xffff)) + pv[2 * e], bf2f((bf16_t)(w[e] >> 16)) + pv[2 * e + 1]);
            v = make_uint4(o[0], o[1], o[2], o[3]);
        }
        if constexpr (EPI == VPF_EPI_BIAS_RESIDUAL) {
            const uint4 rv = res[it];
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
            const uint32_t rr[4] = {rv.x, rv.y, rv.z, rv.w};
            uint32_t o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e)
                o[e] = pack_bf2(bf2f((bf16_t)(w[e] & 0xffff)) + bf2f((bf16_t)(rr[e] & 0xffff)),
                                bf2f((bf16_t)(w[e] >> 16)) + bf2f((bf16_t)(rr[e] >> 16)));
            v = make_uint4(o[0], o[1], o[2], o[3]);
        }
        *reinterpret_cast<uint4*>(C + orow * ldc + n) = v;
    }
}


// ---------------------------------------------------------------------------------------------------------
// Persistent variant: one workgroup per CU walks its XCD's tiles; the (tile, K-step) sequence is one flat
// pipeline, so the DMA of the next tile's first K-tile flies during the current tile's epilogue and no
// workgroup launch / drain separates tiles. Epilogue staged through the free stage of the ring in two
// halves (8 KiB image per wave), each wave reading back only its own image (no block barrier needed).
// Tile assignment: tiles are cut into 8 contiguous chunks, one per XCD group (blocks b, b+8, ... share an
// XCD); the k-th block of a group takes tiles chunk_start + k + r * blocks_in_group, so the blocks running
// together on an XCD work on consecutive tiles (shared A panel / W panels in that XCD's L2).
template <int EPI>
__global__ __launch_bounds__(NTHREADS) void k_gemm_bf16_pers(const bf16_t* __restrict__ A, int lda,
                                                             const bf16_t* __restrict__ W,
                                                             const float* __restrict__ bias,
                                                             const bf16_t* residual,
                                                             const float* __restrict__ pos, int g2,
                                                             const float2* __restrict__ stats,
                                                             const float* __restrict__ colsum,
                                                             bf16_t* C, int ldc, int M, int N, int K, int tiles) {
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid >> 2, wn = wid & 3;
    const int fr = lane & 15, fq = lane >> 4;
    constexpr bool LN = (EPI == VPF_EPI_LN || EPI == VPF_EPI_LN_GELU);

    const int G = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, kx = bid >> 3;
    const int nbx = (G >> 3) + (xcd < (G & 7) ? 1 : 0);
    const int tq = tiles >> 3, tr = tiles & 7;
    const int t_start = xcd < tr ? xcd * (tq + 1) : tr * (tq + 1) + (xcd - tr) * tq;
    const int t_count = tq + (xcd < tr ? 1 : 0);
    const int my_tiles = kx < t_count ? (t_count - kx + nbx - 1) / nbx : 0;
    const int nk = K / BK;
    const int total = my_tiles * nk;
    if (total == 0) return;
    const int tiles_n = (N + BN - 1) / BN;

    // per-lane DMA geometry (tile independent): rows 8g + (lane >> 3) of wave-instructions g = i*8 + wid
    int drow[4], dlch[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        drow[i] = 8 * (i * 8 + wid) + (lane >> 3);
        dlch[i] = ((lane & 7) ^ ((drow[i] >> 1) & 7)) * 16;
    }
    auto tile_of = [&](int r, int& m0, int& n0) {
        const int t = t_start + kx + r * nbx;
        const int tm = t / tiles_n;
        m0 = tm * BM; n0 = (t - tm * tiles_n) * BN;
    };
    auto issue = [&](int st) {
        const int r = st / nk, kt = st - r * nk;
        int m0, n0;
        tile_of(r, m0, n0);
        const char* Ab = reinterpret_cast<const char*>(A) + (size_t)m0 * lda * 2 + (size_t)kt * (BK * 2);
        const char* Bb = reinterpret_cast<const char*>(W) + (size_t)n0 * K * 2 + (size_t)kt * (BK * 2);
        char* la = smem + (st & 1) * STAGE_BYTES;
        char* lb = la + OPERAND_BYTES;
        const int ra_max = M - 1 - m0, rb_max = N - 1 - n0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int g = i * 8 + wid;
            const uint32_t oa = (uint32_t)min(drow[i], ra_max) * (uint32_t)(lda * 2) + (uint32_t)dlch[i];
            const uint32_t ob = (uint32_t)min(drow[i], rb_max) * (uint32_t)(K * 2) + (uint32_t)dlch[i];
            __builtin_amdgcn_global_load_lds((gptr_t)(Ab + oa), (lptr_t)(la + g * 1024), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((gptr_t)(Bb + ob), (lptr_t)(lb + g * 1024), 16, 0, 0);
        }
    };
    float4 bv[4], cv[4];
    float2 rs[8];
    auto load_epi = [&](int m0, int n0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int ng = n0 + wn * 64 + j * 16 + fq * 4;
            bv[j] = ng < N ? *reinterpret_cast<const float4*>(bias + ng) : make_float4(0.f, 0.f, 0.f, 0.f);
            if constexpr (LN) cv[j] = ng < N ? *reinterpret_cast<const float4*>(colsum + ng) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        if constexpr (LN) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int m = m0 + wm * 128 + i * 16 + fr;
                const float2 st = m < M ? stats[m] : make_float2(0.f, 0.f);
                rs[i] = make_float2(st.y, -st.y * st.x);
            }
        }
    };
    f32x4 acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

    int cm0, cn0;
    tile_of(0, cm0, cn0);
    issue(0);
    load_epi(cm0, cn0);
    int kt = 0, r = 0;
    for (int st = 0; st < total; ++st) {
        __syncthreads();   // K-step st landed for every wave; stage (st+1)&1 fully read
        if (st + 1 < total) issue(st + 1);
        const char* la = smem + (st & 1) * STAGE_BYTES;
        const char* lb = la + OPERAND_BYTES;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8 a[8], b[4];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int row = wm * 128 + i * 16 + fr;
                a[i] = *reinterpret_cast<const bf16x8*>(la + row * 128 + (((ks * 4 + fq) ^ ((row >> 1) & 7)) << 4));
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int row = wn * 64 + j * 16 + fr;
                b[j] = *reinterpret_cast<const bf16x8*>(lb + row * 128 + (((ks * 4 + fq) ^ ((row >> 1) & 7)) << 4));
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[j][i], 0, 0, 0);
        }
        if (++kt < nk) continue;
        // ---------------- tile epilogue (stage st&1 is free once every wave is past this barrier) ----------
        kt = 0;
        __syncthreads();
        char* img = smem + (st & 1) * STAGE_BYTES + wid * 8192;
        const int c16 = lane & 7;
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
#pragma unroll
                for (int ii = 0; ii < 4; ++ii) {
                    const int i = hf * 4 + ii;
                    float v0, v1, v2, v3;
                    if constexpr (LN) {
                        v0 = fmaf(rs[i].x, acc[j][i][0], fmaf(rs[i].y, cv[j].x, bv[j].x));
                        v1 = fmaf(rs[i].x, acc[j][i][1], fmaf(rs[i].y, cv[j].y, bv[j].y));
                        v2 = fmaf(rs[i].x, acc[j][i][2], fmaf(rs[i].y, cv[j].z, bv[j].z));
                        v3 = fmaf(rs[i].x, acc[j][i][3], fmaf(rs[i].y, cv[j].w, bv[j].w));
                    } else {
                        v0 = acc[j][i][0] + bv[j].x; v1 = acc[j][i][1] + bv[j].y;
                        v2 = acc[j][i][2] + bv[j].z; v3 = acc[j][i][3] + bv[j].w;
                    }
                    if constexpr (EPI == VPF_EPI_BIAS_GELU || EPI == VPF_EPI_LN_GELU) {
                        const f32x2 g01 = gelu_erf2(f32x2{v0, v1}), g23 = gelu_erf2(f32x2{v2, v3});
                        v0 = g01.x; v1 = g01.y; v2 = g23.x; v3 = g23.y;
                    }
                    const int row = ii * 16 + fr;
                    const int c8 = (j * 4 + fq) ^ (row & 15);
                    *reinterpret_cast<uint2*>(img + row * 128 + c8 * 8) = make_uint2(pack_bf2(v0, v1), pack_bf2(v2, v3));
                }
            }
            uint4 res[8];
            if constexpr (EPI == VPF_EPI_BIAS_RESIDUAL) {
#pragma unroll
                for (int it = 0; it < 8; ++it) {
                    const int m = cm0 + wm * 128 + hf * 64 + it * 8 + (lane >> 3);
                    const int n = cn0 + wn * 64 + c16 * 8;
                    res[it] = (m < M && n < N) ? *reinterpret_cast<const uint4*>(residual + (int64_t)m * ldc + n)
                                               : make_uint4(0, 0, 0, 0);
                }
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int it = 0; it < 8; ++it) {
                const int row = it * 8 + (lane >> 3);
                uint4 v = *reinterpret_cast<const uint4*>(img + row * 128 + ((c16 ^ ((row & 15) >> 1)) * 16));
                if (row & 1) { const uint32_t t0 = v.x, t1 = v.y; v.x = v.z; v.y = v.w; v.z = t0; v.w = t1; }
                const int m = cm0 + wm * 128 + hf * 64 + row;
                const int n = cn0 + wn * 64 + c16 * 8;
                if (m >= M || n >= N) continue;
                int64_t orow = m;
                if constexpr (EPI == VPF_EPI_PATCH) {
                    const int pi = m % g2;
                    orow = (int64_t)(m / g2) * (g2 + 1) + 1 + pi;
                    const float* pr = pos + (int64_t)(1 + pi) * N + n;
                    const float4 p0 = *reinterpret_cast<const float4*>(pr);
                    const float4 p1 = *reinterpret_cast<const float4*>(pr + 4);
                    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
                    const float pv[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
                    uint32_t o[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        o[e] = pack_bf2(bf2f((bf16_t)(w[e] & 0xffff)) + pv[2 * e], bf2f((bf16_t)(w[e] >> 16)) + pv[2 * e + 1]);
                    v = make_uint4(o[0], o[1], o[2], o[3]);
                }
                if constexpr (EPI == VPF_EPI_BIAS_RESIDUAL) {
                    const uint4 rv = res[it];
                    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
                    const uint32_t rr[4] = {rv.x, rv.y, rv.z, rv.w};
                    uint32_t o[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        o[e] = pack_bf2(bf2f((bf16_t)(w[e] & 0xffff)) + bf2f((bf16_t)(rr[e] & 0xffff)),
                                        bf2f((bf16_t)(w[e] >> 16)) + bf2f((bf16_t)(rr[e] >> 16)));
                    v = make_uint4(o[0], o[1], o[2], o[3]);
                }
                *reinterpret_cast<uint4*>(C + orow * ldc + n) = v;
            }
            __builtin_amdgcn_wave_barrier();
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (++r < my_tiles) {
            tile_of(r, cm0, cn0);
            load_epi(cm0, cn0);
        }
    }
}

}  // namespace

#define VPF_GEMM_LAUNCH(E)                                                                                   \
    do {                                                                                                     \
        if (pers)                                                                                            \
            hipLaunchKernelGGL(k_gemm_bf16_pers<E>, pgrid, block, 0, s, A, (int)lda, W, bias, residual, pos,   \
                               patch_rows, reinterpret_cast<const float2*>(row_stats), colsum, C, (int)ldc, m, n, \
                               k, (int)tiles);                                                               \
        else                                                                                                 \
            hipLaunchKernelGGL(k_gemm_bf16<E>, grid, block, 0, s, A, (int)lda, W, bias, residual, pos, patch_rows, \
                               reinterpret_cast<const float2*>(row_stats), colsum, C, (int)ldc, m, n, k, group); \
    } while (0)

// VPF_GEMM_PERSISTENT=1 selects the persistent kernel (one workgroup per CU); the default is one tile per
// workgroup, which measured faster on the ViT-B encoder shapes (5.69 vs 5.43 frames/s, profiles/r1_notes.md).
static int cu_count() {
    static int cached = 0;
    if (!cached) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        cached = n;
    }
    return cached;
}
static int tile_group() {   // VPF_GEMM_GROUP overrides the A-panel group size of the tile order (0 = tm-major)
    static int v = -1;
    if (v < 0) { const char* e = getenv("VPF_GEMM_GROUP"); v = e ? atoi(e) : 8; if (v < 0) v = 0; }
    return v;
}

static bool use_persistent() {
    static int v = -1;
    if (v < 0) { const char* e = getenv("VPF_GEMM_PERSISTENT"); v = (e && e[0] == '1') ? 1 : 0; }
    return v == 1;
}

VPF_API int vpf_gemm_bf16(const uint16_t* A, int64_t lda, const uint16_t* W, const float* bias,
                          const uint16_t* residual, const float* pos, int patch_rows, const float* row_stats,
                          const float* colsum, uint16_t* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                          int epilogue, void* stream) {
    if (M <= 0 || N <= 0 || K <= 0 || K % BK != 0 || N % 8 != 0 || lda < K || lda % 8 != 0 || ldc < N ||
        ldc % 8 != 0)
        return VPF_ERR_ARG;
    if (M > INT32_MAX / 2 || N > 65536 || K > 65536 || lda > INT32_MAX / 2 || ldc > INT32_MAX / 2) return VPF_ERR_ARG;
    if ((uint64_t)BM * (uint64_t)lda * 2 > UINT32_MAX) return VPF_ERR_ARG;
    if (!A || !W || !bias || !C) return VPF_ERR_ARG;
    if (epilogue == VPF_EPI_BIAS_RESIDUAL && !residual) return VPF_ERR_ARG;
    if (epilogue == VPF_EPI_PATCH && (!pos || patch_rows <= 0 || M % patch_rows != 0)) return VPF_ERR_ARG;
    if ((epilogue == VPF_EPI_LN || epilogue == VPF_EPI_LN_GELU) && (!row_stats || !colsum)) return VPF_ERR_ARG;
    // bias / colsum are DMA'd in 16-B pieces, row stats in 4-B pieces
    if (((uintptr_t)bias & 15) || ((uintptr_t)colsum & 15) || ((uintptr_t)row_stats & 7)) return VPF_ERR_ARG;
    const int64_t tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    if (tiles > INT32_MAX) return VPF_ERR_ARG;
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((unsigned)tiles), block(NTHREADS);
    const bool pers = use_persistent();
    const int group = tile_group();
    const dim3 pgrid((unsigned)(tiles < cu_count() ? tiles : cu_count()));
    const int m = (int)M, n = (int)N, k = (int)K;
    switch (epilogue) {
        case VPF_EPI_BIAS: VPF_GEMM_LAUNCH(VPF_EPI_BIAS); break;
        case VPF_EPI_BIAS_GELU: VPF_GEMM_LAUNCH(VPF_EPI_BIAS_GELU); break;
        case VPF_EPI_BIAS_RESIDUAL: VPF_GEMM_LAUNCH(VPF_EPI_BIAS_RESIDUAL); break;
        case VPF_EPI_PATCH: VPF_GEMM_LAUNCH(VPF_EPI_PATCH); break;
        case VPF_EPI_LN: VPF_GEMM_LAUNCH(VPF_EPI_LN); break;
        case VPF_EPI_LN_GELU: VPF_GEMM_LAUNCH(VPF_EPI_LN_GELU); break;
        default: return VPF_ERR_ARG;
    }
    VPF_RETURN_LAUNCH();
}
