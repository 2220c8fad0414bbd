// GEMM lab (design aid, not product): main-loop pipelining variants of the 256x256x64 bf16 MFMA GEMM at the
// ViT-B/16 encoder shapes (M = 4096 x 197 rows), timed in ONE process with interleaved rounds
// (cdna_hip_programming.md §5.4 rule 24) on random data, outputs cross-checked against variant 0.
//
//   V0  product structure: 2-stage LDS ring, one __syncthreads per K-tile, all 8 glds issued up front.
//   V1  V0 + glds issue spread between MFMA groups + s_setprio around MFMA clusters.
//   V2  ping-pong: waves 4-7 run one barrier behind waves 0-3 (one wave of each group per SIMD), so each
//       SIMD alternates a wave in its MFMA segment with a wave in its LDS-read/DMA-issue segment.
//       Segment = 64-deep K-tile; waves 0-3 issue all DMA.
//   V3  ping-pong with 32-deep segments; both groups issue their share of the DMA in their first segment.
//
// Build/run: make -C tools/gemm_lab run   (GPU box)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>
#include <type_traits>

typedef unsigned short bf16_t;
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1); } } while (0)

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int OPB = BM * BK * 2, STB = 2 * OPB, LDSB = 2 * STB;

__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
    __bf16 a = (__bf16)lo, b = (__bf16)hi;
    return (uint32_t)__builtin_bit_cast(unsigned short, a) | ((uint32_t)__builtin_bit_cast(unsigned short, b) << 16);
}

struct Ctx {
    int m0, n0, wid, lane, wm, wn, fr, fq;
    const char* Ablk; const char* Bblk;
};

__device__ __forceinline__ Ctx make_ctx(const bf16_t* A, const bf16_t* W, int M, int N, int K, int wm, int wn) {
    Ctx c;
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    const int lid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    const int tiles_n = (N + BN - 1) / BN;
    const int tm = lid / tiles_n, tn = lid - tm * tiles_n;
    c.m0 = tm * BM; c.n0 = tn * BN;
    c.lane = threadIdx.x & 63;
    c.wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c.wm = wm; c.wn = wn; c.fr = c.lane & 15; c.fq = c.lane >> 4;
    c.Ablk = reinterpret_cast<const char*>(A) + (size_t)c.m0 * K * 2;
    c.Bblk = reinterpret_cast<const char*>(W) + (size_t)c.n0 * K * 2;
    return c;
}

// byte offset (within the block panel) of the 16-B piece lane `lane` moves for wave-instruction g (rows 8g..8g+7)
__device__ __forceinline__ uint32_t dma_off(int g, int lane, int rows_left, int K) {
    const int row = 8 * g + (lane >> 3);
    const int lch = (lane & 7) ^ ((row >> 1) & 7);
    return (uint32_t)min(row, rows_left) * (uint32_t)(K * 2) + (uint32_t)(lch * 16);
}

__device__ __forceinline__ void dma(const char* base, uint32_t off, char* lds) {
    __builtin_amdgcn_global_load_lds((gptr_t)(base + off), (lptr_t)lds, 16, 0, 0);
}

#ifndef LAB_IMM
#define LAB_IMM 1
#endif
__device__ __forceinline__ void read_frags(const char* la, const char* lb, int ks, const Ctx& c, bf16x8 a[8], bf16x8 b[4]) {
#if LAB_IMM
    // rows i*16 + fr share the swizzle term ((fr >> 1) & 7): one base address + i * 2048 immediates
    const int sw = (c.fr >> 1) & 7;
    const char* pa = la + (c.wm * 128 + c.fr) * 128 + (((ks * 4 + c.fq) ^ sw) << 4);
    const char* pb = lb + (c.wn * 64 + c.fr) * 128 + (((ks * 4 + c.fq) ^ sw) << 4);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = *reinterpret_cast<const bf16x8*>(pa + i * 2048);
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const bf16x8*>(pb + j * 2048);
#else
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int row = c.wm * 128 + i * 16 + c.fr;
        a[i] = *reinterpret_cast<const bf16x8*>(la + row * 128 + (((ks * 4 + c.fq) ^ ((row >> 1) & 7)) << 4));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int row = c.wn * 64 + j * 16 + c.fr;
        b[j] = *reinterpret_cast<const bf16x8*>(lb + row * 128 + (((ks * 4 + c.fq) ^ ((row >> 1) & 7)) << 4));
    }
#endif
}

__device__ __forceinline__ void mfma32(f32x4 acc[4][8], const bf16x8 a[8], const bf16x8 b[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i)
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[j][i], 0, 0, 0);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
// G = 1: product GELU (A&S 7.1.26, packed; 2 transcendentals per element)
__device__ __forceinline__ f32x2 gelu_as26(f32x2 x) {
    const f32x2 z = __builtin_elementwise_abs(x) * 0.70710678118654752f;
    const f32x2 den = z * 0.3275911f + 1.0f;
    const f32x2 t = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
    f32x2 p = t * 1.061405429f - 1.453152027f;
    p = p * t + 1.421413741f;
    p = p * t - 0.284496736f;
    p = p * t + 0.254829592f;
    p = p * t;
    const f32x2 ez = z * z * -1.44269504088896341f;
    const f32x2 e = {__builtin_amdgcn_exp2f(ez.x), __builtin_amdgcn_exp2f(ez.y)};
    const f32x2 erf_abs = 1.0f - p * e;
    const f32x2 half = {__builtin_copysignf(0.5f, x.x), __builtin_copysignf(0.5f, x.y)};
    return x * (half * erf_abs + 0.5f);
}
// G = 2: A&S 7.1.28, erfc(z) = (1 + a1 z + ... + a6 z^6)^-16 (|err| <= 3e-7), one rcp per element. The factor
// 2^(1/16) folded into the coefficients makes the reciprocal 0.5 erfc directly: Phi(x) = x<0 ? h : 1-h.
__device__ __forceinline__ f32x2 gelu_as28(f32x2 x) {
    constexpr float c = 1.0442737824274138f;   // 2^(1/16)
    constexpr float s = 0.70710678118654752f;
    const f32x2 z = __builtin_elementwise_abs(x);
    f32x2 p = z * (0.0000430638f * c * s * s * s * s * s * s) + (0.0002765672f * c * s * s * s * s * s);
    p = p * z + (0.0001520143f * c * s * s * s * s);
    p = p * z + (0.0092705272f * c * s * s * s);
    p = p * z + (0.0422820123f * c * s * s);
    p = p * z + (0.0705230784f * c * s);
    p = p * z + c;
    p = p * p; p = p * p; p = p * p; p = p * p;
    const f32x2 h = {__builtin_amdgcn_rcpf(p.x), __builtin_amdgcn_rcpf(p.y)};
    const f32x2 q = 0.5f - h;
    const f32x2 sq = {__builtin_copysignf(q.x, x.x), __builtin_copysignf(q.y, x.y)};
    return x * (sq + 0.5f);
}

template <int G = 0>
__device__ __forceinline__ void epilogue(char* smem, f32x4 acc[4][8], const Ctx& c, const float* bias, bf16_t* C,
                                         int M, int N) {
    __syncthreads();
    char* img = smem + c.wid * 16384;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int ng = c.n0 + c.wn * 64 + j * 16 + c.fq * 4;
        float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ng < N) bv = *reinterpret_cast<const float4*>(bias + ng);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int row = i * 16 + c.fr;
            const int c8 = (j * 4 + c.fq) ^ (row & 15);
            f32x2 v01 = {acc[j][i][0] + bv.x, acc[j][i][1] + bv.y}, v23 = {acc[j][i][2] + bv.z, acc[j][i][3] + bv.w};
            if constexpr (G == 1) { v01 = gelu_as26(v01); v23 = gelu_as26(v23); }
            if constexpr (G == 2) { v01 = gelu_as28(v01); v23 = gelu_as28(v23); }
            *reinterpret_cast<uint2*>(img + row * 128 + c8 * 8) =
                make_uint2(pack_bf2(v01.x, v01.y), pack_bf2(v23.x, v23.y));
        }
    }
    __syncthreads();
    const int c16 = c.lane & 7;
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
        const int row = it * 8 + (c.lane >> 3);
        uint4 v = *reinterpret_cast<const uint4*>(img + row * 128 + ((c16 ^ ((row & 15) >> 1)) * 16));
        if (row & 1) { const uint32_t t0 = v.x, t1 = v.y; v.x = v.z; v.y = v.w; v.z = t0; v.w = t1; }
        const int m = c.m0 + c.wm * 128 + row, n = c.n0 + c.wn * 64 + c16 * 8;
        if (m < M && n < N) *reinterpret_cast<uint4*>(C + (int64_t)m * N + n) = v;
    }
}

// ---------------------------------------------------------------- V0 / V1
template <bool SPREAD, bool SAMEK = false, int G = 0>
__global__ __launch_bounds__(512) void k_v01(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                             const float* __restrict__ bias, bf16_t* C, int M, int N, int K) {
    __shared__ __attribute__((aligned(16))) char smem[LDSB];
    const int wid0 = threadIdx.x >> 6;
    Ctx c = make_ctx(A, W, M, N, K, wid0 >> 2, wid0 & 3);
    uint32_t oa[4], ob[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        oa[i] = dma_off(i * 8 + c.wid, c.lane, M - 1 - c.m0, K);
        ob[i] = dma_off(i * 8 + c.wid, c.lane, N - 1 - c.n0, K);
    }
    f32x4 acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nk = K / BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        dma(c.Ablk, oa[i], smem + (i * 8 + c.wid) * 1024);
        dma(c.Bblk, ob[i], smem + OPB + (i * 8 + c.wid) * 1024);
    }
    for (int kt = 0; kt < nk; ++kt) {
        __syncthreads();
        const char* la = smem + (kt & 1) * STB;
        const char* lb = la + OPB;
        char* na = smem + ((kt + 1) & 1) * STB;
        const uint32_t koff = SAMEK ? 0u : (uint32_t)(kt + 1) * (BK * 2);   // SAMEK: timing probe only
        const bool pre = kt + 1 < nk;
        if (!SPREAD && pre) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                dma(c.Ablk, oa[i] + koff, na + (i * 8 + c.wid) * 1024);
                dma(c.Bblk, ob[i] + koff, na + OPB + (i * 8 + c.wid) * 1024);
            }
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8 a[8], b[4];
            read_frags(la, lb, ks, c, a, b);
            if (SPREAD) __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[j][i], 0, 0, 0);
                if (SPREAD && pre) {
                    const int g = ks * 4 + j;          // 8 DMA pieces over 8 MFMA groups
                    if (g < 4) dma(c.Ablk, oa[g] + koff, na + (g * 8 + c.wid) * 1024);
                    else dma(c.Bblk, ob[g - 4] + koff, na + OPB + ((g - 4) * 8 + c.wid) * 1024);
                }
            }
            if (SPREAD) __builtin_amdgcn_s_setprio(0);
        }
    }
    epilogue<G>(smem, acc, c, bias, C, M, N);
}

// ---------------------------------------------------------------- V2 / V3 ping-pong
// SEG32 = false: one load + one compute segment per 64-deep K-tile, group 0 issues all DMA.
// SEG32 = true : two (32-deep) segment pairs per K-tile, every wave issues its 8 DMA pieces in segment 0.
template <bool SEG32>
__global__ __launch_bounds__(512) void k_pp(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                            const float* __restrict__ bias, bf16_t* C, int M, int N, int K) {
    __shared__ __attribute__((aligned(16))) char smem[LDSB];
    const int wid0 = threadIdx.x >> 6;
    const int grp = wid0 >> 2;
    Ctx c = make_ctx(A, W, M, N, K, grp, wid0 & 3);
    const bool g0 = __builtin_amdgcn_readfirstlane(grp) == 0;
    // DMA pieces of this wave: V2: group-0 wave w moves A pieces {i*4+w} and B pieces {i*4+w}, i < 8;
    //                          V3: every wave moves A/B pieces {i*8+wid}, i < 4 (as V0).
    constexpr int NP = SEG32 ? 4 : 8;
    uint32_t oa[NP], ob[NP];
    int pa[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int g = SEG32 ? (i * 8 + c.wid) : (i * 4 + (c.wid & 3));
        pa[i] = g;
        oa[i] = dma_off(g, c.lane, M - 1 - c.m0, K);
        ob[i] = dma_off(g, c.lane, N - 1 - c.n0, K);
    }
    auto issue = [&](int buf, int kt) {
        char* na = smem + buf * STB;
        const uint32_t koff = (uint32_t)kt * (BK * 2);
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            dma(c.Ablk, oa[i] + koff, na + pa[i] * 1024);
            dma(c.Bblk, ob[i] + koff, na + OPB + pa[i] * 1024);
        }
    };
    f32x4 acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nk = K / BK;
    if (SEG32 || g0) issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                   // #0: tile 0 landed for everyone
    if (!g0) __builtin_amdgcn_s_barrier();         // stagger: group 1 runs one segment behind
    for (int kt = 0; kt < nk; ++kt) {
        const char* la = smem + (kt & 1) * STB;
        const char* lb = la + OPB;
        const bool pre = kt + 1 < nk;
        if (!SEG32) {
            // load segment
            if (g0 && pre) issue((kt + 1) & 1, kt + 1);
            bf16x8 a0[8], b0[4], a1[8], b1[4];
            read_frags(la, lb, 0, c, a0, b0);
            read_frags(la, lb, 1, c, a1, b1);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
            // compute segment
            __builtin_amdgcn_s_setprio(1);
            mfma32(acc, a0, b0);
            mfma32(acc, a1, b1);
            __builtin_amdgcn_s_setprio(0);
            if (g0 && pre) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
        } else {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                if (ks == 0 && pre) issue((kt + 1) & 1, kt + 1);
                bf16x8 a[8], b[4];
                read_frags(la, lb, ks, c, a, b);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                // group 1 retires its DMA at the end of its second load segment; group 0 after its compute
                if (ks == 1 && pre && !g0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_s_setprio(1);
                mfma32(acc, a, b);
                __builtin_amdgcn_s_setprio(0);
                if (ks == 1 && pre && g0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_barrier();
            }
        }
    }
    if (g0) __builtin_amdgcn_s_barrier();          // match group 1's extra barrier
    epilogue(smem, acc, c, bias, C, M, N);
}


// ---------------------------------------------------------------- V4 / V5: 32-deep slice ring
// Ring of R slots, each one 32-deep K-slice of A (256 x 64 B) and B (256 x 64 B) = 32 KiB. 16-B chunk c of row r
// is stored at c ^ F[(r >> 2) & 3], F = {0, 2, 3, 1} (tools/lds_banks.py: conflict-free fragment reads).
// V4 (PP = false): all waves in lockstep, one raw barrier per slice, slices issued R-1 ahead, counted vmcnt.
// V5 (PP = true) : ping-pong groups (waves 4-7 one segment behind); group 0 retires its DMA after its
//                  compute segment, group 1 after its load segment.
__device__ __forceinline__ int fsw(int r) { const int g = (r >> 2) & 3; return (((g ^ (g >> 1)) & 1) << 1) | (g >> 1); }

__device__ __forceinline__ uint32_t dma_off32(int g, int lane, int rows_left, int K) {
    const int row = 16 * g + (lane >> 2);
    const int lch = (lane & 3) ^ fsw(row);
    return (uint32_t)min(row, rows_left) * (uint32_t)(K * 2) + (uint32_t)(lch * 16);
}

__device__ __forceinline__ void read_frags32(const char* la, const char* lb, const Ctx& c, bf16x8 a[8], bf16x8 b[4]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int row = c.wm * 128 + i * 16 + c.fr;
        a[i] = *reinterpret_cast<const bf16x8*>(la + row * 64 + ((c.fq ^ fsw(row)) << 4));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int row = c.wn * 64 + j * 16 + c.fr;
        b[j] = *reinterpret_cast<const bf16x8*>(lb + row * 64 + ((c.fq ^ fsw(row)) << 4));
    }
}

template <int N> __device__ __forceinline__ void wait_vm() {
    if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
}
__device__ __forceinline__ void wait_vm_rt(int n) {   // n = outstanding slices allowed (0..3)
    if (n >= 3) wait_vm<12>(); else if (n == 2) wait_vm<8>(); else if (n == 1) wait_vm<4>(); else wait_vm<0>();
}
__device__ __forceinline__ void bar() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

template <int R, bool PP>
__global__ __launch_bounds__(512) void k_ring(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                              const float* __restrict__ bias, bf16_t* C, int M, int N, int K) {
    constexpr int SLOT = 32768;
    __shared__ __attribute__((aligned(16))) char smem[R * SLOT];
    const int wid0 = threadIdx.x >> 6;
    const int grp = wid0 >> 2;
    Ctx c = make_ctx(A, W, M, N, K, grp, wid0 & 3);
    const bool g1 = PP && __builtin_amdgcn_readfirstlane(grp) == 1;
    uint32_t oa[2], ob[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        oa[i] = dma_off32(i * 8 + c.wid, c.lane, M - 1 - c.m0, K);
        ob[i] = dma_off32(i * 8 + c.wid, c.lane, N - 1 - c.n0, K);
    }
    auto issue = [&](int slot, int sl) {
        char* d = smem + slot * SLOT;
        const uint32_t koff = (uint32_t)sl * 64;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            dma(c.Ablk, oa[i] + koff, d + (i * 8 + c.wid) * 1024);
            dma(c.Bblk, ob[i] + koff, d + 16384 + (i * 8 + c.wid) * 1024);
        }
    };
    f32x4 acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int ns = K / 32;
    for (int sl = 0; sl < R - 1 && sl < ns; ++sl) issue(sl, sl);
    if (!PP) {
        for (int sl = 0; sl < ns; ++sl) {
            wait_vm_rt(min(R - 2, ns - 1 - sl));
            bar();
            if (sl + R - 1 < ns) issue((sl + R - 1) % R, sl + R - 1);
            const char* la = smem + (sl % R) * SLOT;
            bf16x8 a[8], b[4];
            read_frags32(la, la + 16384, c, a, b);
            mfma32(acc, a, b);
        }
    } else {
        wait_vm_rt(min(R - 2, ns - 1));            // slice 0 of every wave
        bar();                                      // #0
        if (g1) bar();                              // stagger
        for (int sl = 0; sl < ns; ++sl) {
            // load segment
            if (sl + R - 1 < ns) issue((sl + R - 1) % R, sl + R - 1);
            const char* la = smem + (sl % R) * SLOT;
            bf16x8 a[8], b[4];
            read_frags32(la, la + 16384, c, a, b);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (g1 && sl + 1 < ns) wait_vm_rt(min(R - 2, ns - 2 - sl));   // my share of slice sl+1
            bar();
            __builtin_amdgcn_s_setprio(1);
            mfma32(acc, a, b);
            __builtin_amdgcn_s_setprio(0);
            if (!g1 && sl + 1 < ns) wait_vm_rt(min(R - 2, ns - 2 - sl));
            bar();
        }
        if (!g1) bar();
    }
    epilogue(smem, acc, c, bias, C, M, N);
}



// ---------------------------------------------------------------- V7: ping-pong + DMA inside compute segments
// Two groups (waves 0-3 / 4-7, one of each per SIMD) one segment apart; segments are 32-deep (12 ds_read_b128
// load segment / 32 MFMA compute segment). Each wave's 8 DMA pieces of a K-tile are issued INSIDE a compute
// segment, one per 4 MFMAs, so the address/TA path streams while the matrix pipe runs:
//   group 0 issues tile k+1 in its first compute segment of tile k, retires it (vmcnt 0) after its second;
//   group 1 issues tile k+1 in its second compute segment of tile k-1, retires it after its second load
//   segment of tile k. Both writes land in the buffer of tile k-1 after every read of it (WAR) and before
//   the first read of tile k+1 (RAW: a barrier separates the retiring wait and the first reader).
template <bool PRIO>
__global__ __launch_bounds__(512) void k_v7(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                            const float* __restrict__ bias, bf16_t* C, int M, int N, int K) {
    __shared__ __attribute__((aligned(16))) char smem[LDSB];
    const int wid0 = threadIdx.x >> 6;
    const int grp = wid0 >> 2;
    Ctx c = make_ctx(A, W, M, N, K, grp, wid0 & 3);
    const bool g1 = __builtin_amdgcn_readfirstlane(grp) == 1;
    uint32_t oa[4], ob[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        oa[i] = dma_off(i * 8 + c.wid, c.lane, M - 1 - c.m0, K);
        ob[i] = dma_off(i * 8 + c.wid, c.lane, N - 1 - c.n0, K);
    }
    auto issue_piece = [&](int buf, int kt, int p) {   // p in [0, 8): A pieces 0..3, B pieces 4..7
        char* na = smem + buf * STB;
        const uint32_t koff = (uint32_t)kt * (BK * 2);
        if (p < 4) dma(c.Ablk, oa[p] + koff, na + (p * 8 + c.wid) * 1024);
        else dma(c.Bblk, ob[p - 4] + koff, na + OPB + ((p - 4) * 8 + c.wid) * 1024);
    };
    f32x4 acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nk = K / BK;
#pragma unroll
    for (int p = 0; p < 8; ++p) issue_piece(0, 0, p);
    if (g1 && nk > 1) {
#pragma unroll
        for (int p = 0; p < 8; ++p) issue_piece(1, 1, p);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar();                                          // #0: tile 0 landed
    if (g1) bar();                                  // stagger
    if (PRIO && g1) __builtin_amdgcn_s_setprio(1);
    for (int kt = 0; kt < nk; ++kt) {
        const char* la = smem + (kt & 1) * STB;
        const char* lb = la + OPB;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            // ---- load segment
            bf16x8 a[8], b[4];
            read_frags(la, lb, ks, c, a, b);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (g1 && ks == 1 && kt + 1 < nk) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // my share of tile kt+1
            bar();
            // ---- compute segment (+ DMA pieces)
            const int dt = g1 ? kt + 2 : kt + 1;          // tile whose pieces this wave streams now
            const bool dma_now = (g1 ? ks == 1 : ks == 0) && dt < nk;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[j][i], 0, 0, 0);
                    if ((i & 3) == 3 && dma_now) issue_piece(dt & 1, dt, j * 2 + (i >> 2));
                }
            }
            if (!g1 && ks == 1 && kt + 1 < nk) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            bar();
        }
    }
    if (PRIO && g1) __builtin_amdgcn_s_setprio(0);
    if (!g1) bar();
    epilogue(smem, acc, c, bias, C, M, N);
}


// ---------------------------------------------------------------- V8: V0 structure on v_mfma_f32_32x32x16_bf16
// Wave tile 128 (m) x 64 (n) = 4 x 2 tiles of 32 x 32 (8 x 16 accumulator VGPRs). Swapped operands: the W
// fragment is the A operand, so D[n][m] has m on the lane and 4 consecutive n per register group.
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ __launch_bounds__(512) void k_v8(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                            const float* __restrict__ bias, bf16_t* C, int M, int N, int K) {
    __shared__ __attribute__((aligned(16))) char smem[LDSB];
    const int wid0 = threadIdx.x >> 6;
    Ctx c = make_ctx(A, W, M, N, K, wid0 >> 2, wid0 & 3);
    const int l32 = c.lane & 31, hh = c.lane >> 5;
    uint32_t oa[4], ob[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        oa[i] = dma_off(i * 8 + c.wid, c.lane, M - 1 - c.m0, K);
        ob[i] = dma_off(i * 8 + c.wid, c.lane, N - 1 - c.n0, K);
    }
    f32x16 acc[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[j][i] = f32x16{};
    const int nk = K / BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        dma(c.Ablk, oa[i], smem + (i * 8 + c.wid) * 1024);
        dma(c.Bblk, ob[i], smem + OPB + (i * 8 + c.wid) * 1024);
    }
    for (int kt = 0; kt < nk; ++kt) {
        __syncthreads();
        const char* la = smem + (kt & 1) * STB;
        const char* lb = la + OPB;
        char* na = smem + ((kt + 1) & 1) * STB;
        const uint32_t koff = (uint32_t)(kt + 1) * (BK * 2);
        if (kt + 1 < nk) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                dma(c.Ablk, oa[i] + koff, na + (i * 8 + c.wid) * 1024);
                dma(c.Bblk, ob[i] + koff, na + OPB + (i * 8 + c.wid) * 1024);
            }
        }
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            bf16x8 a[4], b[2];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = c.wm * 128 + i * 32 + l32;
                a[i] = *reinterpret_cast<const bf16x8*>(la + row * 128 + (((kk * 2 + hh) ^ ((row >> 1) & 7)) << 4));
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int row = c.wn * 64 + j * 32 + l32;
                b[j] = *reinterpret_cast<const bf16x8*>(lb + row * 128 + (((kk * 2 + hh) ^ ((row >> 1) & 7)) << 4));
            }
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    acc[j][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j], a[i], acc[j][i], 0, 0, 0);
        }
    }
    __syncthreads();
    char* img = smem + c.wid * 16384;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int ng = c.n0 + c.wn * 64 + j * 32 + 8 * g + 4 * hh;
            float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
            if (ng < N) bv = *reinterpret_cast<const float4*>(bias + ng);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = i * 32 + l32;
                const int c8 = (j * 8 + 2 * g + hh) ^ (row & 15);
                *reinterpret_cast<uint2*>(img + row * 128 + c8 * 8) =
                    make_uint2(pack_bf2(acc[j][i][4 * g] + bv.x, acc[j][i][4 * g + 1] + bv.y),
                               pack_bf2(acc[j][i][4 * g + 2] + bv.z, acc[j][i][4 * g + 3] + bv.w));
            }
        }
    __builtin_amdgcn_wave_barrier();
    const int c16 = c.lane & 7;
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
        const int row = it * 8 + (c.lane >> 3);
        uint4 v = *reinterpret_cast<const uint4*>(img + row * 128 + ((c16 ^ ((row & 15) >> 1)) * 16));
        if (row & 1) { const uint32_t t0 = v.x, t1 = v.y; v.x = v.z; v.y = v.w; v.z = t0; v.w = t1; }
        const int m = c.m0 + c.wm * 128 + row, n = c.n0 + c.wn * 64 + c16 * 8;
        if (m < M && n < N) *reinterpret_cast<uint4*>(C + (int64_t)m * N + n) = v;
    }
}


// ---------------------------------------------------------------- V9: wave-specialised producer / consumer
// Block tile 256 (m) x 128 (n), BK = 64, 3-stage LDS ring (48 KiB per stage: A 256 rows + B 128 rows).
// Waves 0-3 (one per SIMD) only read LDS and issue MFMAs (wave tile 128 x 64, 128 accumulators, fragments
// double-buffered across the two 32-deep halves of a stage); waves 4-7 only issue LDS-DMA (12 pieces per
// stage each) and retire it with a counted vmcnt. One barrier per K-step: at barrier s, stage s has landed
// (loaders waited before arriving) and stage s-1's slot is free (consumers finished reading it).
constexpr int V9_STAGE = 256 * 128 + 128 * 128;   // 48 KiB
__global__ __launch_bounds__(512) void k_v9(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                            const float* __restrict__ bias, bf16_t* C, int M, int N, int K) {
    __shared__ __attribute__((aligned(16))) char smem[3 * V9_STAGE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool loader = wid >= 4;
    // tile mapping (XCD-aware), BN = 128
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    const int lid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    const int tiles_n = (N + 127) / 128;
    const int tm = lid / tiles_n, tn = lid - tm * tiles_n;
    const int m0 = tm * 256, n0 = tn * 128;
    const char* Ablk = reinterpret_cast<const char*>(A) + (size_t)m0 * K * 2;
    const char* Bblk = reinterpret_cast<const char*>(W) + (size_t)n0 * K * 2;
    const int nk = K / 64;
    const int fr = lane & 15, fq = lane >> 4;
    const int wm = (wid & 3) >> 1, wn = wid & 1;

    if (loader) {
        const int lw = wid - 4;
        uint32_t oa[8], ob[4];
#pragma unroll
        for (int i = 0; i < 8; ++i) oa[i] = dma_off(i * 4 + lw, lane, M - 1 - m0, K);    // A pieces g = i*4 + lw (32)
#pragma unroll
        for (int i = 0; i < 4; ++i) ob[i] = dma_off(i * 4 + lw, lane, N - 1 - n0, K);    // B pieces (16)
        auto issue = [&](int st) {
            char* d = smem + (st % 3) * V9_STAGE;
            const uint32_t koff = (uint32_t)st * 128;
#pragma unroll
            for (int i = 0; i < 8; ++i) dma(Ablk, oa[i] + koff, d + (i * 4 + lw) * 1024);
#pragma unroll
            for (int i = 0; i < 4; ++i) dma(Bblk, ob[i] + koff, d + 32768 + (i * 4 + lw) * 1024);
        };
        issue(0);
        if (nk > 1) issue(1);
        if (nk > 1) asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bar();                                      // B_0: stage 0 landed
        for (int st = 0; st < nk; ++st) {
            if (st + 2 < nk) issue(st + 2);         // slot of stage st-1: free since B_st
            if (st + 1 < nk) {
                if (st + 2 < nk) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                bar();                              // B_{st+1}: stage st+1 landed
            }
        }
        bar();                                      // epilogue barrier (matches consumers)
        return;
    }
    // ---------------- consumers
    f32x4 acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    bar();                                          // B_0
    for (int st = 0; st < nk; ++st) {
        const char* la = smem + (st % 3) * V9_STAGE;
        const char* lb = la + 32768;
        bf16x8 a0[8], b0[4], a1[8], b1[4];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int row = wm * 128 + i * 16 + fr;
            a0[i] = *reinterpret_cast<const bf16x8*>(la + row * 128 + (((0 + fq) ^ ((row >> 1) & 7)) << 4));
            a1[i] = *reinterpret_cast<const bf16x8*>(la + row * 128 + (((4 + fq) ^ ((row >> 1) & 7)) << 4));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = wn * 64 + j * 16 + fr;
            b0[j] = *reinterpret_cast<const bf16x8*>(lb + row * 128 + (((0 + fq) ^ ((row >> 1) & 7)) << 4));
            b1[j] = *reinterpret_cast<const bf16x8*>(lb + row * 128 + (((4 + fq) ^ ((row >> 1) & 7)) << 4));
        }
        mfma32(acc, a0, b0);
        mfma32(acc, a1, b1);
        if (st + 1 < nk) bar();                     // B_{st+1}
    }
    // epilogue (consumers only; loaders wait at the matching barrier so the ring is free)
    bar();
    char* img = smem + wid * 16384;
    {
        Ctx c; c.m0 = m0; c.n0 = n0; c.wid = wid; c.lane = lane; c.wm = wm; c.wn = wn; c.fr = fr; c.fq = fq;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int ng = n0 + wn * 64 + j * 16 + fq * 4;
            float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
            if (ng < N) bv = *reinterpret_cast<const float4*>(bias + ng);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int row = i * 16 + fr;
                const int c8 = (j * 4 + fq) ^ (row & 15);
                *reinterpret_cast<uint2*>(img + row * 128 + c8 * 8) =
                    make_uint2(pack_bf2(acc[j][i][0] + bv.x, acc[j][i][1] + bv.y), pack_bf2(acc[j][i][2] + bv.z, acc[j][i][3] + bv.w));
            }
        }
        __builtin_amdgcn_wave_barrier();
        const int c16 = lane & 7;
#pragma unroll 4
        for (int it = 0; it < 16; ++it) {
            const int row = it * 8 + (lane >> 3);
            uint4 v = *reinterpret_cast<const uint4*>(img + row * 128 + ((c16 ^ ((row & 15) >> 1)) * 16));
            if (row & 1) { const uint32_t t0 = v.x, t1 = v.y; v.x = v.z; v.y = v.w; v.z = t0; v.w = t1; }
            const int m = m0 + wm * 128 + row, n = n0 + wn * 64 + c16 * 8;
            if (m < M && n < N) *reinterpret_cast<uint4*>(C + (int64_t)m * N + n) = v;
        }
    }
}


// ---------------------------------------------------------------- V10: V9 with a mid-stage barrier
// Consumers hold the first-half (k 0-31) fragments of stage s in registers when stage s starts; they issue
// the second-half reads, run the first-half MFMAs, pass barrier X_s (loaders guarantee stage s+1 landed),
// issue stage s+1's first-half reads and run stage s's second-half MFMAs: every LDS read is covered by 32
// MFMAs. A slot is free after X_s for the stage it held (both halves were read between X_{s-1} and X_s).
__global__ __launch_bounds__(512) void k_v10(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                             const float* __restrict__ bias, bf16_t* C, int M, int N, int K) {
    __shared__ __attribute__((aligned(16))) char smem[3 * V9_STAGE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool loader = wid >= 4;
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    const int lid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    const int tiles_n = (N + 127) / 128;
    const int tm = lid / tiles_n, tn = lid - tm * tiles_n;
    const int m0 = tm * 256, n0 = tn * 128;
    const char* Ablk = reinterpret_cast<const char*>(A) + (size_t)m0 * K * 2;
    const char* Bblk = reinterpret_cast<const char*>(W) + (size_t)n0 * K * 2;
    const int nk = K / 64;
    const int fr = lane & 15, fq = lane >> 4;
    const int wm = (wid & 3) >> 1, wn = wid & 1;

    if (loader) {
        const int lw = wid - 4;
        uint32_t oa[8], ob[4];
#pragma unroll
        for (int i = 0; i < 8; ++i) oa[i] = dma_off(i * 4 + lw, lane, M - 1 - m0, K);
#pragma unroll
        for (int i = 0; i < 4; ++i) ob[i] = dma_off(i * 4 + lw, lane, N - 1 - n0, K);
        auto issue = [&](int st) {
            char* d = smem + (st % 3) * V9_STAGE;
            const uint32_t koff = (uint32_t)st * 128;
#pragma unroll
            for (int i = 0; i < 8; ++i) dma(Ablk, oa[i] + koff, d + (i * 4 + lw) * 1024);
#pragma unroll
            for (int i = 0; i < 4; ++i) dma(Bblk, ob[i] + koff, d + 32768 + (i * 4 + lw) * 1024);
        };
        issue(0);
        if (nk > 1) issue(1);
        if (nk > 1) asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bar();                                      // X_-1: stage 0 landed
        for (int st = 0; st + 1 < nk; ++st) {
            // after X_{st-1}: the slot of stage st-1 is free -> stage st+2 (issued for st >= 1; st+2 < nk)
            if (st + 2 < nk) issue(st + 2);      // slot (st+2)%3 held stage st-1 (or is unused for st = 0)
            // X_st must certify stage st+1
            if (st + 2 < nk) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            bar();                                  // X_st
        }
        bar();                                      // epilogue
        return;
    }
    f32x4 acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int sw = (fr >> 1) & 7;
    const int aoff0 = (wm * 128 + fr) * 128 + ((fq ^ sw) << 4), aoff1 = (wm * 128 + fr) * 128 + (((4 + fq) ^ sw) << 4);
    const int boff0 = 32768 + (wn * 64 + fr) * 128 + ((fq ^ sw) << 4), boff1 = 32768 + (wn * 64 + fr) * 128 + (((4 + fq) ^ sw) << 4);
    auto rd = [&](const char* la, int half, bf16x8 a[8], bf16x8 b[4]) {
        const char* pa = la + (half ? aoff1 : aoff0);
        const char* pb = la + (half ? boff1 : boff0);
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = *reinterpret_cast<const bf16x8*>(pa + i * 2048);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const bf16x8*>(pb + j * 2048);
    };
    bar();                                          // X_-1
    bf16x8 a0[8], b0[4], a1[8], b1[4];
    rd(smem, 0, a0, b0);
    for (int st = 0; st < nk; ++st) {
        const char* la = smem + (st % 3) * V9_STAGE;
        rd(la, 1, a1, b1);
        mfma32(acc, a0, b0);
        if (st + 1 < nk) {
            bar();                                  // X_st: stage st+1 landed; stage st-1's slot free
            rd(smem + ((st + 1) % 3) * V9_STAGE, 0, a0, b0);
        }
        mfma32(acc, a1, b1);
    }
    bar();
    char* img = smem + wid * 16384;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int ng = n0 + wn * 64 + j * 16 + fq * 4;
        float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ng < N) bv = *reinterpret_cast<const float4*>(bias + ng);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int row = i * 16 + fr;
            const int c8 = (j * 4 + fq) ^ (row & 15);
            f32x2 v01 = {acc[j][i][0] + bv.x, acc[j][i][1] + bv.y}, v23 = {acc[j][i][2] + bv.z, acc[j][i][3] + bv.w};
            if constexpr (false) { v01 = gelu_as26(v01); v23 = gelu_as26(v23); }
            if constexpr (false) { v01 = gelu_as28(v01); v23 = gelu_as28(v23); }
            *reinterpret_cast<uint2*>(img + row * 128 + c8 * 8) =
                make_uint2(pack_bf2(v01.x, v01.y), pack_bf2(v23.x, v23.y));
        }
    }
    __builtin_amdgcn_wave_barrier();
    const int c16 = lane & 7;
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
        const int row = it * 8 + (lane >> 3);
        uint4 v = *reinterpret_cast<const uint4*>(img + row * 128 + ((c16 ^ ((row & 15) >> 1)) * 16));
        if (row & 1) { const uint32_t t0 = v.x, t1 = v.y; v.x = v.z; v.y = v.w; v.z = t0; v.w = t1; }
        const int m = m0 + wm * 128 + row, n = n0 + wn * 64 + c16 * 8;
        if (m < M && n < N) *reinterpret_cast<uint4*>(C + (int64_t)m * N + n) = v;
    }
}


// ---------------------------------------------------------------- V11: ping-pong with quadrant phases
// Per K-tile 4 phases per wave, each computing one 64 x 32 C-quadrant over K = 64 (16 MFMAs). Quadrant order
// (0,0) (0,1) (1,1) (1,0): fragment reads per load segment 12 / 4 / 8 / 4. DMA pieces of tile k+1 issued
// 3 / 3 / 2 / 0 over the load segments of tile k; group 0 retires after compute phase 3, group 1 after load
// phase 3 (one segment before group 0's first read of tile k+1).
__global__ __launch_bounds__(512) void k_v11(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                             const float* __restrict__ bias, bf16_t* C, int M, int N, int K) {
    __shared__ __attribute__((aligned(16))) char smem[LDSB];
    const int wid0 = threadIdx.x >> 6;
    const int grp = wid0 >> 2;
    Ctx c = make_ctx(A, W, M, N, K, grp, wid0 & 3);
    const bool g1 = __builtin_amdgcn_readfirstlane(grp) == 1;
    uint32_t oa[4], ob[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        oa[i] = dma_off(i * 8 + c.wid, c.lane, M - 1 - c.m0, K);
        ob[i] = dma_off(i * 8 + c.wid, c.lane, N - 1 - c.n0, K);
    }
    auto piece = [&](int buf, int kt, int p) {
        char* na = smem + buf * STB;
        const uint32_t koff = (uint32_t)kt * (BK * 2);
        if (p < 4) dma(c.Ablk, oa[p] + koff, na + (p * 8 + c.wid) * 1024);
        else dma(c.Bblk, ob[p - 4] + koff, na + OPB + ((p - 4) * 8 + c.wid) * 1024);
    };
    const int sw = (c.fr >> 1) & 7;
    const int abase = (c.wm * 128 + c.fr) * 128, bbase = OPB + (c.wn * 64 + c.fr) * 128;
    const int ch0 = (c.fq ^ sw) << 4, ch1 = ((4 + c.fq) ^ sw) << 4;
    f32x4 acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nk = K / BK;
#pragma unroll
    for (int p = 0; p < 8; ++p) piece(0, 0, p);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
    if (g1) bar();
    bf16x8 am[4][2], bn0[2][2], bn1[2][2];   // A rows of one mq half (4 frags x 2 ks), B cols of nq halves
    for (int kt = 0; kt < nk; ++kt) {
        const char* base = smem + (kt & 1) * STB;
        const bool pre = kt + 1 < nk;
        const int nb = (kt + 1) & 1;
#pragma unroll
        for (int ph = 0; ph < 4; ++ph) {
            const int mq = (ph == 0 || ph == 1) ? 0 : 1;
            const int nq = (ph == 0 || ph == 3) ? 0 : 1;
            // ---- load segment
            if (ph == 0 || ph == 2) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    am[i][0] = *reinterpret_cast<const bf16x8*>(base + abase + (mq * 4 + i) * 2048 + ch0);
                    am[i][1] = *reinterpret_cast<const bf16x8*>(base + abase + (mq * 4 + i) * 2048 + ch1);
                }
            }
            if (ph != 2) {
                bf16x8 (&bn)[2][2] = nq ? bn1 : bn0;
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    bn[j][0] = *reinterpret_cast<const bf16x8*>(base + bbase + (nq * 2 + j) * 2048 + ch0);
                    bn[j][1] = *reinterpret_cast<const bf16x8*>(base + bbase + (nq * 2 + j) * 2048 + ch1);
                }
            }
            if (pre) {
                if (ph == 0) { piece(nb, kt + 1, 0); piece(nb, kt + 1, 1); piece(nb, kt + 1, 2); }
                if (ph == 1) { piece(nb, kt + 1, 3); piece(nb, kt + 1, 4); piece(nb, kt + 1, 5); }
                if (ph == 2) { piece(nb, kt + 1, 6); piece(nb, kt + 1, 7); }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (g1 && ph == 3 && pre) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            bar();
            // ---- compute segment: quadrant (mq, nq) over K = 64
            __builtin_amdgcn_s_setprio(1);
            const bf16x8 (&bq)[2][2] = nq ? bn1 : bn0;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        acc[nq * 2 + j][mq * 4 + i] =
                            __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[j][ks], am[i][ks], acc[nq * 2 + j][mq * 4 + i], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
            if (!g1 && ph == 3 && pre) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            bar();
        }
    }
    if (!g1) bar();
    epilogue(smem, acc, c, bias, C, M, N);
}

// ---------------------------------------------------------------- V0 with s_memtime stamps (diagnostic)
__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
__global__ __launch_bounds__(512) void k_v0_stamped(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                    const float* __restrict__ bias, bf16_t* C, int M, int N, int K,
                                                    unsigned long long* dbg) {
    __shared__ __attribute__((aligned(16))) char smem[LDSB];
    const unsigned long long tk0 = stamp();
    const int wid0 = threadIdx.x >> 6;
    Ctx c = make_ctx(A, W, M, N, K, wid0 >> 2, wid0 & 3);
    uint32_t oa[4], ob[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        oa[i] = dma_off(i * 8 + c.wid, c.lane, M - 1 - c.m0, K);
        ob[i] = dma_off(i * 8 + c.wid, c.lane, N - 1 - c.n0, K);
    }
    f32x4 acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nk = K / BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        dma(c.Ablk, oa[i], smem + (i * 8 + c.wid) * 1024);
        dma(c.Bblk, ob[i], smem + OPB + (i * 8 + c.wid) * 1024);
    }
    unsigned long long s_wait = 0, s_issue = 0, s_comp = 0, s_first = 0;
    const unsigned long long tloop = stamp();
    for (int kt = 0; kt < nk; ++kt) {
        const unsigned long long t0 = stamp();
        __syncthreads();
        const unsigned long long t1 = stamp();
        const char* la = smem + (kt & 1) * STB;
        const char* lb = la + OPB;
        char* na = smem + ((kt + 1) & 1) * STB;
        const uint32_t koff = (uint32_t)(kt + 1) * (BK * 2);
        if (kt + 1 < nk) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                dma(c.Ablk, oa[i] + koff, na + (i * 8 + c.wid) * 1024);
                dma(c.Bblk, ob[i] + koff, na + OPB + (i * 8 + c.wid) * 1024);
            }
        }
        const unsigned long long t2 = stamp();
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8 a[8], b[4];
            read_frags(la, lb, ks, c, a, b);
            mfma32(acc, a, b);
        }
        // make the stamp wait for the MFMAs: consume one accumulator
        asm volatile("" :: "v"(acc[3][7]));
        const unsigned long long t3 = stamp();
        s_wait += t1 - t0; s_issue += t2 - t1; s_comp += t3 - t2;
        if (kt == 0) s_first = t1 - tloop;
    }
    const unsigned long long tep = stamp();
    epilogue(smem, acc, c, bias, C, M, N);
    const unsigned long long tend = stamp();
    if (c.lane == 0) {
        unsigned long long* d = dbg + ((size_t)blockIdx.x * 8 + c.wid) * 8;
        d[0] = tloop - tk0; d[1] = s_wait; d[2] = s_issue; d[3] = s_comp; d[4] = tend - tep; d[5] = tend - tk0;
        d[6] = s_first; d[7] = tk0;
    }
}

__global__ __launch_bounds__(512) void k_v10s(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                             const float* __restrict__ bias, bf16_t* C, int M, int N, int K,
                                             unsigned long long* dbg) {
    __shared__ __attribute__((aligned(16))) char smem[3 * V9_STAGE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool loader = wid >= 4;
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    const int lid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    const int tiles_n = (N + 127) / 128;
    const int tm = lid / tiles_n, tn = lid - tm * tiles_n;
    const int m0 = tm * 256, n0 = tn * 128;
    const char* Ablk = reinterpret_cast<const char*>(A) + (size_t)m0 * K * 2;
    const char* Bblk = reinterpret_cast<const char*>(W) + (size_t)n0 * K * 2;
    const int nk = K / 64;
    const int fr = lane & 15, fq = lane >> 4;
    const int wm = (wid & 3) >> 1, wn = wid & 1;

    if (loader) {
        const int lw = wid - 4;
        uint32_t oa[8], ob[4];
#pragma unroll
        for (int i = 0; i < 8; ++i) oa[i] = dma_off(i * 4 + lw, lane, M - 1 - m0, K);
#pragma unroll
        for (int i = 0; i < 4; ++i) ob[i] = dma_off(i * 4 + lw, lane, N - 1 - n0, K);
        auto issue = [&](int st) {
            char* d = smem + (st % 3) * V9_STAGE;
            const uint32_t koff = (uint32_t)st * 128;
#pragma unroll
            for (int i = 0; i < 8; ++i) dma(Ablk, oa[i] + koff, d + (i * 4 + lw) * 1024);
#pragma unroll
            for (int i = 0; i < 4; ++i) dma(Bblk, ob[i] + koff, d + 32768 + (i * 4 + lw) * 1024);
        };
        issue(0);
        if (nk > 1) issue(1);
        if (nk > 1) asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bar();                                      // X_-1: stage 0 landed
        unsigned long long t_issue = 0, t_vm = 0, t_bar = 0;
        for (int st = 0; st + 1 < nk; ++st) {
            const unsigned long long t0 = stamp();
            if (st + 2 < nk) issue(st + 2);
            const unsigned long long t1 = stamp();
            if (st + 2 < nk) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned long long t2 = stamp();
            bar();
            const unsigned long long t3 = stamp();
            t_issue += t1 - t0; t_vm += t2 - t1; t_bar += t3 - t2;
        }
        if (lane == 0) { unsigned long long* d = dbg + ((size_t)blockIdx.x * 8 + wid) * 4; d[0] = t_issue; d[1] = t_vm; d[2] = t_bar; d[3] = 1; }
        bar();                                      // epilogue
        return;
    }
    f32x4 acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int sw = (fr >> 1) & 7;
    const int aoff0 = (wm * 128 + fr) * 128 + ((fq ^ sw) << 4), aoff1 = (wm * 128 + fr) * 128 + (((4 + fq) ^ sw) << 4);
    const int boff0 = 32768 + (wn * 64 + fr) * 128 + ((fq ^ sw) << 4), boff1 = 32768 + (wn * 64 + fr) * 128 + (((4 + fq) ^ sw) << 4);
    auto rd = [&](const char* la, int half, bf16x8 a[8], bf16x8 b[4]) {
        const char* pa = la + (half ? aoff1 : aoff0);
        const char* pb = la + (half ? boff1 : boff0);
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = *reinterpret_cast<const bf16x8*>(pa + i * 2048);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const bf16x8*>(pb + j * 2048);
    };
    bar();                                          // X_-1
    bf16x8 a0[8], b0[4], a1[8], b1[4];
    rd(smem, 0, a0, b0);
    unsigned long long t_m1 = 0, t_bar = 0, t_m2 = 0;
    for (int st = 0; st < nk; ++st) {
        const char* la = smem + (st % 3) * V9_STAGE;
        const unsigned long long t0 = stamp();
        rd(la, 1, a1, b1);
        mfma32(acc, a0, b0);
        asm volatile("" :: "v"(acc[3][7]));
        const unsigned long long t1 = stamp();
        if (st + 1 < nk) {
            bar();
            rd(smem + ((st + 1) % 3) * V9_STAGE, 0, a0, b0);
        }
        const unsigned long long t2 = stamp();
        mfma32(acc, a1, b1);
        asm volatile("" :: "v"(acc[3][7]));
        const unsigned long long t3 = stamp();
        t_m1 += t1 - t0; t_bar += t2 - t1; t_m2 += t3 - t2;
    }
    if (lane == 0) { unsigned long long* d = dbg + ((size_t)blockIdx.x * 8 + wid) * 4; d[0] = t_m1; d[1] = t_bar; d[2] = t_m2; d[3] = 0; }
    bar();
    char* img = smem + wid * 16384;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int ng = n0 + wn * 64 + j * 16 + fq * 4;
        float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ng < N) bv = *reinterpret_cast<const float4*>(bias + ng);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int row = i * 16 + fr;
            const int c8 = (j * 4 + fq) ^ (row & 15);
            f32x2 v01 = {acc[j][i][0] + bv.x, acc[j][i][1] + bv.y}, v23 = {acc[j][i][2] + bv.z, acc[j][i][3] + bv.w};
            if constexpr (false) { v01 = gelu_as26(v01); v23 = gelu_as26(v23); }
            if constexpr (false) { v01 = gelu_as28(v01); v23 = gelu_as28(v23); }
            *reinterpret_cast<uint2*>(img + row * 128 + c8 * 8) =
                make_uint2(pack_bf2(v01.x, v01.y), pack_bf2(v23.x, v23.y));
        }
    }
    __builtin_amdgcn_wave_barrier();
    const int c16 = lane & 7;
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
        const int row = it * 8 + (lane >> 3);
        uint4 v = *reinterpret_cast<const uint4*>(img + row * 128 + ((c16 ^ ((row & 15) >> 1)) * 16));
        if (row & 1) { const uint32_t t0 = v.x, t1 = v.y; v.x = v.z; v.y = v.w; v.z = t0; v.w = t1; }
        const int m = m0 + wm * 128 + row, n = n0 + wn * 64 + c16 * 8;
        if (m < M && n < N) *reinterpret_cast<uint4*>(C + (int64_t)m * N + n) = v;
    }
}


// ---------------------------------------------------------------- host

// ---------------------------------------------------------------- V12: occupancy 2
// 256x128x32 tile, 4 waves (each the same 128x64 sub-tile as V0), 2-stage ring of 64-B rows (16-B chunk c of
// row r at c ^ F[(r >> 2) & 3], conflict-free per tools/lds_banks.py), 64 KiB LDS -> two workgroups per CU,
// so one workgroup's barrier waits and epilogue overlap the other's MFMA stream.
constexpr int V12_A = 256 * 64, V12_STAGE = 384 * 64;   // bytes
__device__ __forceinline__ int f64sw(int r) { return (0x1E0 >> (2 * ((r >> 2) & 3))) & 3; }   // F = {0,2,3,1}
__device__ __forceinline__ uint32_t dma_off_r64(int g, int lane, int rows_left, int K) {
    const int row = 16 * g + (lane >> 2);
    const int ch = (lane & 3) ^ f64sw(row);
    return (uint32_t)min(row, rows_left) * (uint32_t)(K * 2) + (uint32_t)(ch * 16);
}
template <int G = 0>
__global__ __launch_bounds__(256, 2) void k_v12(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                const float* __restrict__ bias, bf16_t* C, int M, int N, int K) {
    __shared__ __attribute__((aligned(16))) char smem[65536];
    Ctx c;
    {
        const int nwg = gridDim.x, bid = blockIdx.x;
        const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
        const int lid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
        const int tiles_n = (N + 127) / 128;
        const int tm = lid / tiles_n, tn = lid - tm * tiles_n;
        c.m0 = tm * 256; c.n0 = tn * 128;
        c.lane = threadIdx.x & 63;
        c.wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        c.wm = c.wid >> 1; c.wn = c.wid & 1; c.fr = c.lane & 15; c.fq = c.lane >> 4;
        c.Ablk = reinterpret_cast<const char*>(A) + (size_t)c.m0 * K * 2;
        c.Bblk = reinterpret_cast<const char*>(W) + (size_t)c.n0 * K * 2;
    }
    uint32_t oa[4], ob[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) oa[i] = dma_off_r64(i * 4 + c.wid, c.lane, M - 1 - c.m0, K);
#pragma unroll
    for (int i = 0; i < 2; ++i) ob[i] = dma_off_r64(i * 4 + c.wid, c.lane, N - 1 - c.n0, K);
    f32x4 acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nk = K / 32;
#pragma unroll
    for (int i = 0; i < 4; ++i) dma(c.Ablk, oa[i], smem + (i * 4 + c.wid) * 1024);
#pragma unroll
    for (int i = 0; i < 2; ++i) dma(c.Bblk, ob[i], smem + V12_A + (i * 4 + c.wid) * 1024);
    const int sw = f64sw(c.fr);
    const int aoff = (c.wm * 128 + c.fr) * 64 + ((c.fq ^ sw) << 4);
    const int boff = V12_A + (c.wn * 64 + c.fr) * 64 + ((c.fq ^ sw) << 4);
    for (int kt = 0; kt < nk; ++kt) {
        __syncthreads();
        const char* st = smem + (kt & 1) * V12_STAGE;
        char* ns = smem + ((kt + 1) & 1) * V12_STAGE;
        if (kt + 1 < nk) {
            const uint32_t koff = (uint32_t)(kt + 1) * 64;
#pragma unroll
            for (int i = 0; i < 4; ++i) dma(c.Ablk, oa[i] + koff, ns + (i * 4 + c.wid) * 1024);
#pragma unroll
            for (int i = 0; i < 2; ++i) dma(c.Bblk, ob[i] + koff, ns + V12_A + (i * 4 + c.wid) * 1024);
        }
        bf16x8 a[8], b[4];
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = *reinterpret_cast<const bf16x8*>(st + aoff + i * 1024);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const bf16x8*>(st + boff + j * 1024);
        mfma32(acc, a, b);
    }
    epilogue<G>(smem, acc, c, bias, C, M, N);
}


// ---------------------------------------------------------------- V13: 4 waves x 128x128 (1 wave / SIMD)
// hipBLASLt's gfx950 bf16 kernel shape (MT256x256x64, 256 threads, 130 KB LDS): each wave owns a 128x128
// sub-tile (8 x 8 16x16x32 MFMA tiles, 256 fp32 accumulators in the unified VGPR/AGPR file), which halves
// the LDS fragment reads per MFMA versus 8 waves of 128x64. Same 2-stage glds ring and swizzle as V0.
template <int G = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void k_v13(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W, const float* __restrict__ bias, bf16_t* C,
           int M, int N, int K) {
    __shared__ __attribute__((aligned(16))) char smem[LDSB];
    const int wid0 = threadIdx.x >> 6;
    Ctx c = make_ctx(A, W, M, N, K, wid0 >> 1, wid0 & 1);
    uint32_t oa[8], ob[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        oa[i] = dma_off(i * 4 + c.wid, c.lane, M - 1 - c.m0, K);
        ob[i] = dma_off(i * 4 + c.wid, c.lane, N - 1 - c.n0, K);
    }
    f32x4 acc[8][8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nk = K / BK;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        dma(c.Ablk, oa[i], smem + (i * 4 + c.wid) * 1024);
        dma(c.Bblk, ob[i], smem + OPB + (i * 4 + c.wid) * 1024);
    }
    const int sw = (c.fr >> 1) & 7;
    for (int kt = 0; kt < nk; ++kt) {
        __syncthreads();
        const char* la = smem + (kt & 1) * STB;
        const char* lb = la + OPB;
        char* na = smem + ((kt + 1) & 1) * STB;
        if (kt + 1 < nk) {
            const uint32_t koff = (uint32_t)(kt + 1) * (BK * 2);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                dma(c.Ablk, oa[i] + koff, na + (i * 4 + c.wid) * 1024);
                dma(c.Bblk, ob[i] + koff, na + OPB + (i * 4 + c.wid) * 1024);
            }
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const char* pa = la + (c.wm * 128 + c.fr) * 128 + (((ks * 4 + c.fq) ^ sw) << 4);
            const char* pb = lb + (c.wn * 128 + c.fr) * 128 + (((ks * 4 + c.fq) ^ sw) << 4);
            bf16x8 a[8], b[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) a[i] = *reinterpret_cast<const bf16x8*>(pa + i * 2048);
#pragma unroll
            for (int j = 0; j < 8; ++j) b[j] = *reinterpret_cast<const bf16x8*>(pb + j * 2048);
#pragma unroll
            for (int j = 0; j < 8; ++j)
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[j][i], 0, 0, 0);
        }
    }
    // epilogue: two 128x64 halves per wave, 16 KiB image each (4 waves x 2 x 16 KiB = the whole ring)
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        char* img = smem + c.wid * 32768 + h * 16384;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int ng = c.n0 + c.wn * 128 + h * 64 + j * 16 + c.fq * 4;
            float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
            if (ng < N) bv = *reinterpret_cast<const float4*>(bias + ng);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int row = i * 16 + c.fr;
                const int c8 = (j * 4 + c.fq) ^ (row & 15);
                f32x2 v01 = {acc[h * 4 + j][i][0] + bv.x, acc[h * 4 + j][i][1] + bv.y};
                f32x2 v23 = {acc[h * 4 + j][i][2] + bv.z, acc[h * 4 + j][i][3] + bv.w};
                if constexpr (G == 1) { v01 = gelu_as26(v01); v23 = gelu_as26(v23); }
                if constexpr (G == 2) { v01 = gelu_as28(v01); v23 = gelu_as28(v23); }
                *reinterpret_cast<uint2*>(img + row * 128 + c8 * 8) = make_uint2(pack_bf2(v01.x, v01.y), pack_bf2(v23.x, v23.y));
            }
        }
    }
    __syncthreads();
    const int c16 = c.lane & 7;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const char* img = smem + c.wid * 32768 + h * 16384;
#pragma unroll 4
        for (int it = 0; it < 16; ++it) {
            const int row = it * 8 + (c.lane >> 3);
            uint4 v = *reinterpret_cast<const uint4*>(img + row * 128 + ((c16 ^ ((row & 15) >> 1)) * 16));
            if (row & 1) { const uint32_t t0 = v.x, t1 = v.y; v.x = v.z; v.y = v.w; v.z = t0; v.w = t1; }
            const int m = c.m0 + c.wm * 128 + row, n = c.n0 + c.wn * 128 + h * 64 + c16 * 8;
            if (m < M && n < N) *reinterpret_cast<uint4*>(C + (int64_t)m * N + n) = v;
        }
    }
}


// ---------------------------------------------------------------- V14: V13 software-pipelined
// 4 waves x 128x128, 4-slot ring of 32-deep slices (A 256 x 64 B + B 256 x 64 B = 32 KiB per slot, chunk
// swizzle F = {0,2,3,1}). Iteration t: one barrier (slice t+1 landed for every wave; slot of slice t-1 free),
// then 64 MFMAs on the fragments of slice t (registers) interleaved with the 16 fragment reads of slice t+1
// and the 8 DMA pieces of slice t+3. DMA runs 3 slices (~3 K MFMA cycles) ahead; counted vmcnt.
template <int G = 0, int INTERLEAVE = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void k_v14(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W, const float* __restrict__ bias, bf16_t* C,
           int M, int N, int K) {
    constexpr int SLOT = 32768;
    __shared__ __attribute__((aligned(16))) char smem[4 * SLOT];
    const int wid0 = threadIdx.x >> 6;
    Ctx c = make_ctx(A, W, M, N, K, wid0 >> 1, wid0 & 1);
    uint32_t oa[4], ob[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        oa[i] = dma_off32(i * 4 + c.wid, c.lane, M - 1 - c.m0, K);
        ob[i] = dma_off32(i * 4 + c.wid, c.lane, N - 1 - c.n0, K);
    }
    f32x4 acc[8][8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int ns = K / 32;
    auto issue_piece = [&](int sl, int p) {       // p = 0..7: A pieces 0-3, B pieces 4-7
        char* d = smem + (sl & 3) * SLOT;
        const uint32_t koff = (uint32_t)sl * 64;
        if (p < 4) dma(c.Ablk, oa[p] + koff, d + (p * 4 + c.wid) * 1024);
        else dma(c.Bblk, ob[p - 4] + koff, d + 16384 + ((p - 4) * 4 + c.wid) * 1024);
    };
    const int sw = fsw(c.fr);
    const int aoff = (c.wm * 128 + c.fr) * 64 + ((c.fq ^ sw) << 4);
    const int boff = 16384 + (c.wn * 128 + c.fr) * 64 + ((c.fq ^ sw) << 4);
    for (int sl = 0; sl < 3 && sl < ns; ++sl)
#pragma unroll
        for (int p = 0; p < 8; ++p) issue_piece(sl, p);
    bf16x8 a0[8], b0[8], a1[8], b1[8];
    if (ns >= 3) wait_vm<16>(); else if (ns == 2) wait_vm<8>(); else wait_vm<0>();
    bar();
#pragma unroll
    for (int i = 0; i < 8; ++i) a0[i] = *reinterpret_cast<const bf16x8*>(smem + aoff + i * 1024);
#pragma unroll
    for (int j = 0; j < 8; ++j) b0[j] = *reinterpret_cast<const bf16x8*>(smem + boff + j * 1024);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

    // Branch-free body (one basic block per slice, so the sched_group_barrier interleave applies): the
    // fragment reads of "slice ns" read a stale slot (never used); DMA slices past the end re-fetch slice
    // ns-1 into a slot nobody reads again; so every iteration waits vmcnt(8) (= the slice issued one
    // iteration ago may still fly).
    auto step = [&](int t, bf16x8 (&ac)[8], bf16x8 (&bc)[8], bf16x8 (&an)[8], bf16x8 (&bn)[8]) {
        wait_vm<8>();
        bar();
        const char* ls = smem + ((t + 1) & 3) * SLOT;
        char* dd = smem + ((t + 3) & 3) * SLOT;
        const uint32_t koff = (uint32_t)min(t + 3, ns - 1) * 64;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
                acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bc[j], ac[i], acc[j][i], 0, 0, 0);
            an[j] = *reinterpret_cast<const bf16x8*>(ls + aoff + j * 1024);
            bn[j] = *reinterpret_cast<const bf16x8*>(ls + boff + j * 1024);
            if (j < 4) dma(c.Ablk, oa[j] + koff, dd + (j * 4 + c.wid) * 1024);
            else dma(c.Bblk, ob[j - 4] + koff, dd + 16384 + ((j - 4) * 4 + c.wid) * 1024);
            if constexpr (INTERLEAVE) {
                __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
    for (int t = 0; t < ns; t += 2) {
        step(t, a0, b0, a1, b1);
        step(t + 1, a1, b1, a0, b0);
    }
    // epilogue: two 128x64 halves per wave, 16 KiB image each (4 waves x 2 x 16 KiB = the whole ring)
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        char* img = smem + c.wid * 32768 + h * 16384;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int ng = c.n0 + c.wn * 128 + h * 64 + j * 16 + c.fq * 4;
            float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
            if (ng < N) bv = *reinterpret_cast<const float4*>(bias + ng);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int row = i * 16 + c.fr;
                const int c8 = (j * 4 + c.fq) ^ (row & 15);
                f32x2 v01 = {acc[h * 4 + j][i][0] + bv.x, acc[h * 4 + j][i][1] + bv.y};
                f32x2 v23 = {acc[h * 4 + j][i][2] + bv.z, acc[h * 4 + j][i][3] + bv.w};
                if constexpr (G == 1) { v01 = gelu_as26(v01); v23 = gelu_as26(v23); }
                if constexpr (G == 2) { v01 = gelu_as28(v01); v23 = gelu_as28(v23); }
                *reinterpret_cast<uint2*>(img + row * 128 + c8 * 8) = make_uint2(pack_bf2(v01.x, v01.y), pack_bf2(v23.x, v23.y));
            }
        }
    }
    __syncthreads();
    const int c16 = c.lane & 7;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const char* img = smem + c.wid * 32768 + h * 16384;
#pragma unroll 4
        for (int it = 0; it < 16; ++it) {
            const int row = it * 8 + (c.lane >> 3);
            uint4 v = *reinterpret_cast<const uint4*>(img + row * 128 + ((c16 ^ ((row & 15) >> 1)) * 16));
            if (row & 1) { const uint32_t t0 = v.x, t1 = v.y; v.x = v.z; v.y = v.w; v.z = t0; v.w = t1; }
            const int m = c.m0 + c.wm * 128 + row, n = c.n0 + c.wn * 128 + h * 64 + c16 * 8;
            if (m < M && n < N) *reinterpret_cast<uint4*>(C + (int64_t)m * N + n) = v;
        }
    }
}


// ---------------------------------------------------------------- V15: persistent V14
// grid = min(tiles, CUs). Each workgroup walks tiles lid, lid + nwg, ... (XCD-grouped lid: the workgroups of
// one XCD work on consecutive tiles). The slice stream is continuous across tiles: the DMA cursor runs 3
// slices ahead and crosses into the next tile during the current tile's last slices, so no pipeline fill
// per tile. DMA = buffer_load ... lds through a per-slice buffer resource (base = panel + k offset,
// num_records = bytes left in the panel): rows past M / N are hardware OOB -> zeros, so per-lane offsets are
// tile-invariant; a cursor past the last tile gets num_records = 0 (no traffic). First slice of a tile
// runs its MFMAs with C = 0 (no accumulator reset). Epilogue stores 8-B pieces straight from the
// accumulators; bias rides the DMA stream one tile ahead into a double-buffered LDS aux region.
__device__ unsigned long long* g_dbg15;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void bdma(__amdgpu_buffer_rsrc_t r, uint32_t voff, char* lds) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}
template <int G = 0, bool STAMP = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void k_v15(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W, const float* __restrict__ bias, bf16_t* C,
           int M, int N, int K) {
    unsigned long long st_wait = 0, st_body = 0, st_epi = 0, st_t0 = 0;
    constexpr int SLOT = 32768;
    __shared__ __attribute__((aligned(16))) char smem[4 * SLOT + 2048];
    char* aux = smem + 4 * SLOT;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wid >> 1, wn = wid & 1, fr = lane & 15, fq = lane >> 4;
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    const int lid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    const int tiles_n = (N + 255) / 256, ntiles = ((M + 255) / 256) * tiles_n;
    const int ns = K / 32;
    uint32_t vo[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = 16 * (i * 4 + wid) + (lane >> 2);
        vo[i] = (uint32_t)row * (uint32_t)(K * 2) + (uint32_t)((((lane & 3) ^ fsw(row))) * 16);
    }
    // DMA cursor (wave-uniform)
    int dtile = lid, dt = 0;
    uint32_t dslot = 0;
    auto dma_slice = [&]() {
        const bool ok = dtile < ntiles;
        const int tm = dtile / tiles_n, tn = dtile - tm * tiles_n;
        const uint32_t ra = ok ? (uint32_t)min(M - tm * 256, 256) * (uint32_t)(K * 2) - (uint32_t)dt * 64 : 0u;
        const uint32_t rb = ok ? (uint32_t)min(N - tn * 256, 256) * (uint32_t)(K * 2) - (uint32_t)dt * 64 : 0u;
        const __amdgpu_buffer_rsrc_t rA = mk_rsrc(A + ((size_t)(ok ? tm : 0) * 256 * K + dt * 32), ra);
        const __amdgpu_buffer_rsrc_t rB = mk_rsrc(W + ((size_t)(ok ? tn : 0) * 256 * K + dt * 32), rb);
        char* d = smem + (dslot & 3) * SLOT;
#pragma unroll
        for (int i = 0; i < 4; ++i) bdma(rA, vo[i], d + (i * 4 + wid) * 1024);
#pragma unroll
        for (int i = 0; i < 4; ++i) bdma(rB, vo[i], d + 16384 + (i * 4 + wid) * 1024);
        ++dslot;
        ++dt;
        if (dt == ns) { dt = 0; dtile += nwg; }
    };
    auto dma_bias = [&](int tile, int buf) {   // wave 0 only
        const bool ok = tile < ntiles;
        const int tn = ok ? tile % tiles_n : 0;
        const __amdgpu_buffer_rsrc_t rb = mk_rsrc(bias + tn * 256, ok ? (uint32_t)min(N - tn * 256, 256) * 4u : 0u);
        bdma(rb, (uint32_t)lane * 16, aux + buf * 1024);
    };
    if (lid >= ntiles) return;
    if (wid == 0) dma_bias(lid, 0);
    dma_slice(); dma_slice(); dma_slice();
    const int sw = fsw(fr);
    const int aoff = (wm * 128 + fr) * 64 + ((fq ^ sw) << 4);
    const int boff = 16384 + (wn * 128 + fr) * 64 + ((fq ^ sw) << 4);
    bf16x8 a0[8], b0[8], a1[8], b1[8];
    wait_vm<16>();
    bar();
#pragma unroll
    for (int i = 0; i < 8; ++i) a0[i] = *reinterpret_cast<const bf16x8*>(smem + aoff + i * 1024);
#pragma unroll
    for (int j = 0; j < 8; ++j) b0[j] = *reinterpret_cast<const bf16x8*>(smem + boff + j * 1024);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    f32x4 acc[8][8];
    uint32_t s = 0;   // global compute slice
    auto step = [&](auto first, bf16x8 (&ac)[8], bf16x8 (&bc)[8], bf16x8 (&an)[8], bf16x8 (&bn)[8]) {
        unsigned long long ta = 0, tb = 0;
        if constexpr (STAMP) ta = __builtin_amdgcn_s_memtime();
        wait_vm<8>();
        bar();
        if constexpr (STAMP) tb = __builtin_amdgcn_s_memtime();
        const char* ls = smem + ((s + 1) & 3) * SLOT;
        // the 8 DMA pieces of the cursor slice, spread over the 8 MFMA groups
        const bool ok = dtile < ntiles;
        const int tm = dtile / tiles_n, tn = dtile - tm * tiles_n;
        const uint32_t ra = ok ? (uint32_t)min(M - tm * 256, 256) * (uint32_t)(K * 2) - (uint32_t)dt * 64 : 0u;
        const uint32_t rb = ok ? (uint32_t)min(N - tn * 256, 256) * (uint32_t)(K * 2) - (uint32_t)dt * 64 : 0u;
        const __amdgpu_buffer_rsrc_t rA = mk_rsrc(A + ((size_t)(ok ? tm : 0) * 256 * K + dt * 32), ra);
        const __amdgpu_buffer_rsrc_t rB = mk_rsrc(W + ((size_t)(ok ? tn : 0) * 256 * K + dt * 32), rb);
        char* dd = smem + (dslot & 3) * SLOT;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if constexpr (decltype(first)::value)
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bc[j], ac[i], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                else
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bc[j], ac[i], acc[j][i], 0, 0, 0);
            }
            an[j] = *reinterpret_cast<const bf16x8*>(ls + aoff + j * 1024);
            bn[j] = *reinterpret_cast<const bf16x8*>(ls + boff + j * 1024);
            if (j < 4) bdma(rA, vo[j], dd + (j * 4 + wid) * 1024);
            else bdma(rB, vo[j - 4], dd + 16384 + ((j - 4) * 4 + wid) * 1024);
            __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
        ++dslot;
        ++dt;
        if (dt == ns) { dt = 0; dtile += nwg; }
        ++s;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (STAMP) { const unsigned long long tc = __builtin_amdgcn_s_memtime(); st_wait += tb - ta; st_body += tc - tb; }
    };
    using T = std::true_type;
    using F = std::false_type;
    int k = 0;
    for (int tile = lid; tile < ntiles; tile += nwg, ++k) {
        step(T{}, a0, b0, a1, b1);
        step(F{}, a1, b1, a0, b0);
        for (int t = 2; t < ns; t += 2) {
            step(F{}, a0, b0, a1, b1);
            step(F{}, a1, b1, a0, b0);
        }
        unsigned long long te0 = 0;
        if constexpr (STAMP) te0 = __builtin_amdgcn_s_memtime();
        // next tile's bias (lands long before its epilogue; older than the slices waited on -> counted)
        if (wid == 0) dma_bias(tile + nwg, (k + 1) & 1);
        // epilogue of this tile, straight from the accumulators
        const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
        const char* ab = aux + (k & 1) * 1024;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int nl = wn * 128 + j * 16 + fq * 4;
            const float4 bv = *reinterpret_cast<const float4*>(ab + nl * 4);
            const int n = tn * 256 + nl;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int m = tm * 256 + wm * 128 + i * 16 + fr;
                f32x2 v01 = {acc[j][i][0] + bv.x, acc[j][i][1] + bv.y};
                f32x2 v23 = {acc[j][i][2] + bv.z, acc[j][i][3] + bv.w};
                if constexpr (G == 1) { v01 = gelu_as26(v01); v23 = gelu_as26(v23); }
                if constexpr (G == 2) { v01 = gelu_as28(v01); v23 = gelu_as28(v23); }
                if (m < M && n < N)
                    *reinterpret_cast<uint2*>(C + (int64_t)m * N + n) = make_uint2(pack_bf2(v01.x, v01.y), pack_bf2(v23.x, v23.y));
            }
        }
        if constexpr (STAMP) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); st_epi += __builtin_amdgcn_s_memtime() - te0; }
    }
    if constexpr (STAMP) {
        if (lane == 0) {
            unsigned long long* o = g_dbg15 + ((size_t)blockIdx.x * 4 + wid) * 4;
            o[0] = st_wait; o[1] = st_body; o[2] = st_epi; o[3] = (unsigned long long)k;
        }
    }
    wait_vm<0>();   // outstanding (OOB / zero) DMAs must land before the workgroup's LDS is released
}

static void fill_bf16(std::vector<bf16_t>& v, float scale, unsigned seed) {
    std::mt19937 g(seed);
    std::uniform_real_distribution<float> d(-1.f, 1.f);
    for (auto& x : v) {
        float f = d(g) * scale;
        uint32_t u; memcpy(&u, &f, 4);
        x = (bf16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
    }
}

typedef void (*kfn)(const bf16_t*, const bf16_t*, const float*, bf16_t*, int, int, int);

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 3;
    const char* shape_filter = argc > 2 ? argv[2] : "";      // e.g. "fc2"
    const char* var_filter = argc > 3 ? argv[3] : "";        // e.g. "V0,V3"
    const bool check = argc <= 4 || atoi(argv[4]) != 0;
    struct Shape { const char* name; int M, N, K; };
    const int Mtok = 4096 * 197;
    Shape shapes[] = {{"qkv", Mtok, 2304, 768}, {"proj", Mtok, 768, 768}, {"fc1", Mtok, 3072, 768},
                      {"fc2", Mtok, 768, 3072}, {"small_qkv", 16384, 2304, 768}, {"small_fc2", 65536, 768, 3072}};
    struct Var { const char* name; kfn f; };
    Var vars[] = {{"V0", k_v01<false>}, {"V1", k_v01<true>}, {"V2", k_pp<false>}, {"V3", k_pp<true>},
                  {"V4r4", k_ring<4, false>}, {"V4r5", k_ring<5, false>}, {"V5r4", k_ring<4, true>},
                  {"V5r5", k_ring<5, true>}, {"V7", k_v7<false>}, {"V7p", k_v7<true>},
                  {"V0samek", k_v01<false, true>}, {"V8", k_v8}, {"V9", k_v9}, {"V10", k_v10}, {"V11", k_v11},
                  {"V0g1", k_v01<false, false, 1>}, {"V0g2", k_v01<false, false, 2>}, {"V12", k_v12<0>},
                  {"V12g1", k_v12<1>}, {"V12g2", k_v12<2>},
                  {"V13", k_v13<0>}, {"V13g2", k_v13<2>},
                  {"V14", k_v14<0, 1>}, {"V14n", k_v14<0, 0>}, {"V14g2", k_v14<2, 1>},
                  {"V15", k_v15<0>}, {"V15g2", k_v15<2>}};
    const int NV = sizeof(vars) / sizeof(vars[0]);
    size_t maxA = 0, maxW = 0, maxC = 0;
    for (auto& s : shapes) {
        maxA = std::max(maxA, (size_t)s.M * s.K); maxW = std::max(maxW, (size_t)s.N * s.K);
        maxC = std::max(maxC, (size_t)s.M * s.N);
    }
    std::vector<bf16_t> hA(maxA), hW(maxW);
    fill_bf16(hA, 1.0f, 1); fill_bf16(hW, 0.05f, 2);
    if (getenv("LAB_ZERO")) { std::fill(hA.begin(), hA.end(), 0); std::fill(hW.begin(), hW.end(), 0); }
    std::vector<float> hb(4096, 0.01f);
    bf16_t *dA, *dW, *dC0, *dC;
    float* db;
    CHECK(hipMalloc(&dA, maxA * 2)); CHECK(hipMalloc(&dW, maxW * 2));
    CHECK(hipMalloc(&dC0, maxC * 2)); CHECK(hipMalloc(&dC, maxC * 2)); CHECK(hipMalloc(&db, 4096 * 4));
    CHECK(hipMemcpy(dA, hA.data(), maxA * 2, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dW, hW.data(), maxW * 2, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(db, hb.data(), 4096 * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    std::vector<bf16_t> ref(maxC), got(maxC);
    for (auto& s : shapes) {
        if (shape_filter[0] && !strstr(shape_filter, s.name)) continue;
        const int tiles = ((s.M + BM - 1) / BM) * ((s.N + BN - 1) / BN);
        const int tiles128 = ((s.M + BM - 1) / BM) * ((s.N + 127) / 128);
        auto grid_of = [&](int v) { return dim3((strcmp(vars[v].name, "V9") == 0 || strcmp(vars[v].name, "V10") == 0 ||
                                                  strncmp(vars[v].name, "V12", 3) == 0) ? tiles128
                                               : strncmp(vars[v].name, "V15", 3) == 0 ? std::min(tiles, 256) : tiles); };
        auto block_of = [&](int v) { return dim3(strncmp(vars[v].name, "V12", 3) == 0 || strncmp(vars[v].name, "V13", 3) == 0 ||
                                                          strncmp(vars[v].name, "V14", 3) == 0 ||
                                                          strncmp(vars[v].name, "V15", 3) == 0 ? 256 : 512); };
        const double flop = 2.0 * s.M * (double)s.N * s.K;
        std::vector<std::vector<float>> ms(NV);
        auto on = [&](int v) { return !var_filter[0] || strstr(var_filter, vars[v].name); };
        if (check) {
        // correctness vs V0
        hipLaunchKernelGGL(vars[0].f, dim3(tiles), dim3(512), 0, 0, dA, dW, db, dC0, s.M, s.N, s.K);
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(ref.data(), dC0, (size_t)s.M * s.N * 2, hipMemcpyDeviceToHost));
        for (int v = 1; v < NV; ++v) {
            CHECK(hipMemset(dC, 0, (size_t)s.M * s.N * 2));
            hipLaunchKernelGGL(vars[v].f, grid_of(v), block_of(v), 0, 0, dA, dW, db, dC, s.M, s.N, s.K);
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy(got.data(), dC, (size_t)s.M * s.N * 2, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t i = 0; i < (size_t)s.M * s.N; ++i) bad += got[i] != ref[i];
            printf("%s %s mismatches vs V0: %zu\n", s.name, vars[v].name, bad);
        }
        }
        for (int r = 0; r < rounds; ++r)
            for (int v = 0; v < NV; ++v) {
                if (!on(v)) { ms[v].push_back(0.f); continue; }
                CHECK(hipEventRecord(e0, 0));
                for (int it = 0; it < 3; ++it)
                    hipLaunchKernelGGL(vars[v].f, grid_of(v), block_of(v), 0, 0, dA, dW, db, dC, s.M, s.N, s.K);
                CHECK(hipEventRecord(e1, 0));
                CHECK(hipEventSynchronize(e1));
                float t; CHECK(hipEventElapsedTime(&t, e0, e1));
                ms[v].push_back(t / 3);
            }
        for (int v = 0; v < NV; ++v) {
            std::sort(ms[v].begin(), ms[v].end());
            const float med = ms[v][ms[v].size() / 2];
            printf("%-5s %-3s M=%d N=%d K=%d  median %.3f ms  %.1f TFLOP/s  (min %.3f)\n", s.name, vars[v].name, s.M, s.N,
                   s.K, med, flop / (med * 1e-3) / 1e12, ms[v][0]);
        }
        fflush(stdout);
    }
    if (getenv("LAB_STAMPS15")) {
        for (auto& sh : shapes) {
            if (shape_filter[0] && !strstr(shape_filter, sh.name)) continue;
            const int tiles = ((sh.M + 255) / 256) * ((sh.N + 255) / 256);
            const int g = std::min(tiles, 256);
            unsigned long long* dbg;
            CHECK(hipMalloc(&dbg, (size_t)g * 16 * 8));
            CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_dbg15), &dbg, sizeof(dbg)));
            for (int rep = 0; rep < 2; ++rep)
                hipLaunchKernelGGL((k_v15<0, true>), dim3(g), dim3(256), 0, 0, dA, dW, db, dC, sh.M, sh.N, sh.K);
            CHECK(hipDeviceSynchronize());
            std::vector<unsigned long long> h((size_t)g * 16);
            CHECK(hipMemcpy(h.data(), dbg, h.size() * 8, hipMemcpyDeviceToHost));
            double w = 0, b = 0, e = 0, nt = 0;
            for (int i = 0; i < g * 4; ++i) { w += h[i * 4]; b += h[i * 4 + 1]; e += h[i * 4 + 2]; nt += h[i * 4 + 3]; }
            const double slices = nt * (sh.K / 32);
            printf("V15 stamps %s: per slice wait+bar %.0f body %.0f | per tile epilogue %.0f (memtime units; tiles/wave %.1f)\n",
                   sh.name, w / slices, b / slices, e / nt, nt / (g * 4));
            CHECK(hipFree(dbg));
        }
    }
    if (getenv("LAB_STAMPS10")) {
        for (auto& s : shapes) {
            if (shape_filter[0] && !strstr(shape_filter, s.name)) continue;
            const int tiles = ((s.M + BM - 1) / BM) * ((s.N + 127) / 128);
            unsigned long long* dbg;
            CHECK(hipMalloc(&dbg, (size_t)tiles * 32 * 8));
            for (int rep = 0; rep < 2; ++rep)
                hipLaunchKernelGGL(k_v10s, dim3(tiles), dim3(512), 0, 0, dA, dW, db, dC, s.M, s.N, s.K, dbg);
            CHECK(hipDeviceSynchronize());
            std::vector<unsigned long long> h((size_t)tiles * 32);
            CHECK(hipMemcpy(h.data(), dbg, h.size() * 8, hipMemcpyDeviceToHost));
            double c[3] = {0}, l[3] = {0};
            for (int t = 0; t < tiles; ++t)
                for (int w = 0; w < 8; ++w)
                    for (int k = 0; k < 3; ++k) (w < 4 ? c : l)[k] += (double)h[((size_t)t * 8 + w) * 4 + k];
            const double nb = (double)tiles * 4 * (s.K / 64);
            printf("V10 stamps %s per stage (cycles): consumer mfma1(+rd) %.0f bar(+rd0) %.0f mfma2 %.0f | loader issue %.0f vmwait %.0f bar %.0f\n",
                   s.name, c[0] / nb, c[1] / nb, c[2] / nb, l[0] / nb, l[1] / nb, l[2] / nb);
            CHECK(hipFree(dbg));
        }
    }
    if (getenv("LAB_STAMPS")) {
        for (auto& s : shapes) {
            if (shape_filter[0] && !strstr(shape_filter, s.name)) continue;
            const int tiles = ((s.M + BM - 1) / BM) * ((s.N + BN - 1) / BN);
            unsigned long long* dbg;
            CHECK(hipMalloc(&dbg, (size_t)tiles * 64 * 8));
            for (int rep = 0; rep < 2; ++rep)
                hipLaunchKernelGGL(k_v0_stamped, dim3(tiles), dim3(512), 0, 0, dA, dW, db, dC, s.M, s.N, s.K, dbg);
            CHECK(hipDeviceSynchronize());
            std::vector<unsigned long long> h((size_t)tiles * 64);
            CHECK(hipMemcpy(h.data(), dbg, h.size() * 8, hipMemcpyDeviceToHost));
            double acc[8] = {0};
            for (int t = 0; t < tiles; ++t)
                for (int w = 0; w < 8; ++w)
                    for (int k = 0; k < 7; ++k) acc[k] += (double)h[((size_t)t * 8 + w) * 8 + k];
            const double nb = (double)tiles * 8;
            printf("stamps %s (per wave, avg cycles): prologue %.0f | loop: wait %.0f issue %.0f compute %.0f (first wait %.0f) | epilogue %.0f | total %.0f\n",
                   s.name, acc[0] / nb, acc[1] / nb, acc[2] / nb, acc[3] / nb, acc[6] / nb, acc[4] / nb, acc[5] / nb);
            CHECK(hipFree(dbg));
        }
    }
    return 0;
}
