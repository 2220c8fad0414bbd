// bf16 GEMM with fused epilogues for the ViT encoder.
//
//   C[M][N] = epi( A[M][K] . W[N][K]^T ),  bf16 operands, fp32 accumulation on MFMA.
//
// Design (gfx950; MI355X_MICROARCH.md / cdna_hip_programming.md §5):
//  * 256x256 output tile, BK = 64, 512 threads = 8 waves laid out 2 (M) x 4 (N); each wave owns a
//    128 (M) x 64 (N) sub-tile = 8 x 4 fragments of v_mfma_f32_16x16x32_bf16 (128 accumulator VGPRs).
//  * Operands are staged HBM/L2 -> LDS by global_load_lds_dwordx4 (LDS-DMA, 1 KiB per wave-instruction,
//    no VGPR round trip). Ring: 3 A K-tiles + 2 B K-tiles (5 x 32 KiB = the whole 160 KiB of LDS): the
//    activation panel (the operand that misses L2) is prefetched 2 K-tiles ahead, the L2-hot weights 1.
//    The LDS image is lane-linear; bank conflicts of the fragment reads (ds_read_b128) are removed by
//    XOR-swizzling the per-lane SOURCE address: 16-B chunk c of row r lives at physical chunk
//    c ^ ((r >> 1) & 7) (tools/lds_banks.py: conflict-free for every 16-lane group).
//  * One raw s_barrier per K-step behind a counted vmcnt (the next A K-tile stays in flight across it);
//    right after it, the DMA for B(t+1) and A(t+2) is issued and flies while the 64 MFMAs per wave run.
//  * MFMA operands are "swapped" (W fragment as A, activation fragment as B) so the accumulator holds
//    D[n][m]: each lane owns 4 consecutive output columns of one row. Epilogue: bias (+ GELU, gelu_sig2)
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
// epilogue operands: bias (1 KiB) | colsum (1 KiB) | row statistics (up to AUX_PARTS planes of 2 KiB).
// 16 planes (D = 1024) do not fit next to bias / colsum: the deep ring then lands them in a second free A
// slot at the last K-step (wide path).
constexpr int AUX_PARTS = 15;
constexpr int MAX_PARTS = 16;
constexpr int AUX_BYTES = 2048 + AUX_PARTS * 2048;

typedef const __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

typedef float f32x2 __attribute__((ext_vector_type(2)));

// bf16-path GELU, two values at a time: x * sigmoid(x (a + b x^2)) = x / (1 + 2^(x (c1 + c2 x^2))), with (a, b)
// the minimax fit to the exact-erf GELU over [-10, 10] (a = 1.6003142, b = 0.0694018; the tanh form's
// a = 2 sqrt(2/pi), b = 0.044715 a has 4.7e-4): max |error| 2.7e-4, an eighth of the bf16 half-ulp at |y| = 1.
// 9 instructions per pair (3 packed mul/fma, 2 v_exp_f32, 1 packed add, 2 v_rcp_f32, 1 packed mul) against
// ~21 + hazard nops for gelu_erf2. x -> -inf: 2^(+inf) = inf, rcp = 0, y = -0; x -> +inf: y = x.
__device__ __forceinline__ f32x2 gelu_sig2(f32x2 x) {
    constexpr float L2E = 1.4426950408889634f;
    constexpr float c1 = -1.6003141571059616f * L2E, c2 = -0.06940178687219423f * L2E;
    const f32x2 q = (x * x) * c2 + c1;
    const f32x2 t = x * q;
    const f32x2 d = f32x2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + 1.0f;
    return x * f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}


// Epilogue of one wave's 128 (M) x 64 (N) sub-tile. `img` is this wave's private 16 KiB of LDS (free of any
// operand the other waves still read), `aux` the epilogue-operand region (bias | colsum at column offset
// wn*64 of the tile, row statistics at row offset wm*128). Bias / LN-fold / GELU in fp32 on the
// accumulators, bf16 pack, 8-B writes into an XOR-swizzled image, then 16-B coalesced row stores (+ residual
// / position-embedding adds on the packed values). `stats_out` (may be null): for the producers of the
// residual stream (EPI_BIAS_RESIDUAL, EPI_PATCH) the per-row {sum, sumsq} of the stored bf16 values over the
// wave's 64 columns go to plane n0/64 + wn (plane stride stats_rows rows): each lane's 8-value partial is
// parked in the image row it was just read from, then each lane sums the 8 partials of two rows and stores
// them with one 16-B store; no cross-wave step.
template <int EPI>
__device__ __forceinline__ void store_wave_tile(char* img, const char* aux, const f32x4 (&acc)[4][8], int wm, int wn,
                                                int m0, int n0, int lane, const bf16_t* residual,
                                                const float* __restrict__ pos, int g2, bf16_t* C, int ldc, int M,
                                                int N, float* stats_out, int stats_rows) {
    constexpr bool LN = (EPI == VPF_EPI_LN || EPI == VPF_EPI_LN_GELU);
    const int fr = lane & 15, fq = lane >> 4;
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
                v01 = gelu_sig2(v01);
                v23 = gelu_sig2(v23);
            }
            const int row = i * 16 + fr;              // row within the wave's 128-row image
            const int c8 = (j * 4 + fq) ^ (row & 15);  // swizzled 8-B chunk
            *reinterpret_cast<uint2*>(img + row * 128 + c8 * 8) =
                make_uint2(pack_bf2(v01.x, v01.y), pack_bf2(v23.x, v23.y));
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
    constexpr bool PROD = (EPI == VPF_EPI_BIAS_RESIDUAL || EPI == VPF_EPI_PATCH);
    __builtin_amdgcn_wave_barrier();   // the image is private to this wave: LDS ops of one wave stay in order
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int row = it * 8 + (lane >> 3);
        uint4 v = *reinterpret_cast<const uint4*>(img + row * 128 + ((c16 ^ ((row & 15) >> 1)) * 16));
        if (row & 1) { const uint32_t t0 = v.x, t1 = v.y; v.x = v.z; v.y = v.w; v.z = t0; v.w = t1; }
        const int m = m0 + wm * 128 + row;
        const int n = n0 + wn * 64 + c16 * 8;
        const bool ok = m < M && n < N;
        int64_t orow = m;
        if constexpr (EPI == VPF_EPI_PATCH) {
            const int pi = m % g2;
            orow = (int64_t)(m / g2) * (g2 + 1) + 1 + pi;
            const float* pr = pos + (int64_t)(1 + pi) * N + min(n, N - 8);
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
        if constexpr (PROD) {
            if (stats_out != nullptr) {   // wave-uniform
                // {sum, sumsq} of the lane's 8 stored values
                // v_dot2_f32_bf16 on the packed pairs: sum = dot(w, (1, 1)), sumsq = dot(w, w) (bf16 products are
                // exact in fp32)
                typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
                const uint32_t w[4] = {v.x, v.y, v.z, v.w};
                const bf16x2_t one2 = __builtin_bit_cast(bf16x2_t, 0x3F803F80u);
                float s1 = 0.f, s2 = 0.f;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const bf16x2_t pr = __builtin_bit_cast(bf16x2_t, w[e]);
                    s1 = __builtin_amdgcn_fdot2_f32_bf16(pr, one2, s1, false);
                    s2 = __builtin_amdgcn_fdot2_f32_bf16(pr, pr, s2, false);
                }
                if (!ok) { s1 = 0.f; s2 = 0.f; }
                // the lane's partial goes back into the image row it was just read from (8 B at c16 * 8; the
                // whole row was read by this same instruction above and LDS ops of one wave stay in order)
                *reinterpret_cast<float2*>(img + row * 128 + c16 * 8) = make_float2(s1, s2);
            }
        }
        if (ok) *reinterpret_cast<uint4*>(C + orow * ldc + n) = v;
    }
    if constexpr (PROD) {
        const int nb = n0 + wn * 64;
        if (stats_out != nullptr && nb < N) {   // wave-uniform
            __builtin_amdgcn_wave_barrier();
            // rows 2*lane, 2*lane+1: the 8 lane partials of each (64 B at the row start)
            float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 u0 = *reinterpret_cast<const float4*>(img + (2 * lane) * 128 + q * 16);
                const float4 u1 = *reinterpret_cast<const float4*>(img + (2 * lane + 1) * 128 + q * 16);
                t.x += u0.x + u0.z; t.y += u0.y + u0.w;
                t.z += u1.x + u1.z; t.w += u1.y + u1.w;
            }
            float* plane = stats_out + (int64_t)(nb >> 6) * stats_rows * 2;
            const int m = m0 + wm * 128 + 2 * lane;
            if constexpr (EPI == VPF_EPI_PATCH) {
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const int me = m + e;
                    if (me < M) {
                        const int64_t orow = (int64_t)(me / g2) * (g2 + 1) + 1 + me % g2;
                        *reinterpret_cast<float2*>(plane + orow * 2) = e ? make_float2(t.z, t.w) : make_float2(t.x, t.y);
                    }
                }
            } else {
                if (m + 1 < M) *reinterpret_cast<float4*>(plane + (int64_t)m * 2) = t;
                else if (m < M) *reinterpret_cast<float2*>(plane + (int64_t)m * 2) = make_float2(t.x, t.y);
            }
        }
    }
}

template <int EPI, bool DEEP, bool WIDE = false>
__global__ __launch_bounds__(NTHREADS) void k_gemm_bf16(const bf16_t* __restrict__ A, int lda,
                                                        const bf16_t* __restrict__ W,
                                                        const float* __restrict__ bias,
                                                        const bf16_t* residual,
                                                        const float* __restrict__ pos, int g2,
                                                        const float2* __restrict__ stats,
                                                        const float* __restrict__ colsum,
                                                        bf16_t* C, int ldc, int M, int N, int K, int group,
                                                        int stats_parts, float ln_eps, float* stats_out,
                                                        int stats_rows) {
    // DEEP: A ring of 3 K-tiles (A prefetched 2 K-tiles ahead: the activation panel is the operand that
    // misses L2), B ring of 2 (weights stay L2-hot); 5 x 32 KiB = all 160 KiB of LDS, and the epilogue
    // operands go into the A slot no K-tile uses any more (slot nk % 3, DMA'd at K-tile max(nk-2, 0)).
    // !DEEP: the 2-stage A+B ring (2 x 64 KiB + 4 KiB aux), kept for A/B timing (vpf_gemm_tune).
    constexpr int SMEM = DEEP ? 5 * OPERAND_BYTES : LDS_BYTES + AUX_BYTES;
    static_assert(AUX_BYTES <= OPERAND_BYTES, "aux region must fit the free A slot of the deep ring");
    __shared__ __attribute__((aligned(16))) char smem[SMEM];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);

    // ---- XCD-aware bijective block -> tile remap ----
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    const int lid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    // Grouped order inside each XCD's contiguous lid range: groups of `group` A row-panels; within a group
    // the A panel index runs fastest, so the ~32 tiles an XCD has in flight cover ~group A panels x
    // 32/group W panels and both stay in that XCD's L2 (tm-major order re-fetched a 393 KB W panel per
    // tile on FC1: FETCH_SIZE 14.8 GB/launch, profiles/r1_notes.md). group = 0: plain tm-major. Default 4
    // (4 A x 8 W panels in flight per XCD: ~11-12 distinct K-slices per K-step for 32 tiles, the minimum of
    // a + b at a*b = 32): sweep 2..24 in profiles/r1_gemm_lab/group_sweep.txt, 4 best or tied on all shapes.
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
    auto stage_a = [&](int kt) {   // DEEP: A K-tile kt -> A slot kt % 3
        char* la = smem + (kt % 3) * OPERAND_BYTES;
        const uint32_t koff = (uint32_t)kt * (BK * 2);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds((gptr_t)(Ablk + offA[i] + koff), (lptr_t)(la + (i * 8 + wid) * 1024), 16, 0, 0);
    };
    auto stage_b = [&](int kt) {   // DEEP: B K-tile kt -> B slot kt & 1
        char* lb = smem + (3 + (kt & 1)) * OPERAND_BYTES;
        const uint32_t koff = (uint32_t)kt * (BK * 2);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds((gptr_t)(Bblk + offB[i] + koff), (lptr_t)(lb + (i * 8 + wid) * 1024), 16, 0, 0);
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
    const int nk = K / BK;
    char* aux = DEEP ? smem + (nk % 3) * OPERAND_BYTES : smem + LDS_BYTES;
    // stats_parts == 0: one {mean, rstd} plane; else stats_parts {sum, sumsq} planes of M rows each. A
    // plane's 256-row slice is 2 KiB = two 16-B-per-lane pieces (M even, 16-B aligned base), dealt round-robin
    // over the 8 waves (12 planes: 3 pieces per wave instead of 12 4-B pieces).
    constexpr bool LN_ = (EPI == VPF_EPI_LN || EPI == VPF_EPI_LN_GELU);
    constexpr bool wide = DEEP && LN_ && WIDE;   // host: only for stats_parts > AUX_PARTS
    char* planes_lds = wide ? smem + ((nk + 1) % 3) * OPERAND_BYTES : aux + 2048;
    auto load_planes = [&](char* dst) {
        const float* sd = reinterpret_cast<const float*>(stats);
        const int planes = stats_parts > 0 ? stats_parts : 1;
        if ((M & 1) == 0 && ((uintptr_t)sd & 15) == 0) {
            for (int pc = wid; pc < 2 * planes; pc += 8) {
                const int p = pc >> 1, hf = pc & 1;
                __builtin_amdgcn_global_load_lds(
                    (gptr_t)(sd + (int64_t)p * 2 * M + min(2 * m0 + hf * 256 + lane * 4, 2 * M - 4)),
                    (lptr_t)(dst + p * 2048 + hf * 1024), 16, 0, 0);
            }
        } else {
            for (int p = 0; p < planes; ++p)
                __builtin_amdgcn_global_load_lds(
                    (gptr_t)(sd + (int64_t)p * 2 * M + min(2 * m0 + wid * 64 + lane, 2 * M - 1)),
                    (lptr_t)(dst + p * 2048 + wid * 256), 4, 0, 0);
        }
    };
    auto load_aux = [&]() {
        if (wid == 0)
            __builtin_amdgcn_global_load_lds((gptr_t)(bias + min(n0 + lane * 4, N - 4)), (lptr_t)aux, 16, 0, 0);
        if constexpr (LN) {
            if (wid == 1)
                __builtin_amdgcn_global_load_lds((gptr_t)(colsum + min(n0 + lane * 4, N - 4)), (lptr_t)(aux + 1024), 16,
                                                 0, 0);
            if (!wide) load_planes(aux + 2048);
        }
    };
    if constexpr (!DEEP) {
        load_aux();
        stage(0, 0);
    } else {
        stage_a(0);
        stage_b(0);
        if (nk > 1) stage_a(1);
    }
    for (int kt = 0; kt < nk; ++kt) {
        const char* la;
        const char* lb;
        if constexpr (!DEEP) {
            __syncthreads();   // vmcnt(0) + barrier: tile kt landed for every wave; tile kt-1 fully read
            if (kt + 1 < nk) stage((kt + 1) & 1, kt + 1);
            la = smem + (kt & 1) * STAGE_BYTES;
            lb = la + OPERAND_BYTES;
        } else {
            // issue order: A0 B0 A1 | per K-tile t: B(t+1) A(t+2). A(kt), B(kt) are older than everything but
            // A(kt+1) (4 pieces per wave) until the last two K-tiles, where the tail is B / aux only.
            if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if (kt + 1 < nk) stage_b(kt + 1);
            if (kt + 2 < nk) stage_a(kt + 2);
            if (kt == (nk >= 2 ? nk - 2 : 0)) load_aux();
            if (wide && kt == nk - 1) load_planes(planes_lds);   // slot of A(nk-2): free after this barrier
            la = smem + (kt % 3) * OPERAND_BYTES;
            lb = smem + (3 + (kt & 1)) * OPERAND_BYTES;
        }
        // both 32-deep halves' fragments are read up front (24 ds_read_b128): the second half's reads
        // complete under the first half's 32 MFMAs instead of stalling between them
        bf16x8 a[2][8], b[2][4];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int row = wn * 64 + j * 16 + fr;
                const int ch = (ks * 4 + fq) ^ ((row >> 1) & 7);
                b[ks][j] = *reinterpret_cast<const bf16x8*>(lb + row * 128 + ch * 16);
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int row = wm * 128 + i * 16 + fr;
                const int ch = (ks * 4 + fq) ^ ((row >> 1) & 7);
                a[ks][i] = *reinterpret_cast<const bf16x8*>(la + row * 128 + ch * 16);
            }
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[ks][j], a[ks][i], acc[j][i], 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 24, 0);   // the 24 fragment reads first
        __builtin_amdgcn_sched_group_barrier(0x008, 64, 0);   // then the 64 MFMAs (counted lgkmcnt waits)
    }

    // ---------------- epilogue ----------------
    if constexpr (LN) {
        // statistics planes -> {mean, rstd} once per row (in place over plane 0, which only this thread
        // reads), instead of in each of the 4 waves that share the row; the aux DMA landed before the last
        // K-step's barrier
        if constexpr (wide) {   // the planes DMA'd at the last K-step must land for every wave
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
        if (stats_parts > 0 && tid < BM) {
            float sm = 0.f, sq = 0.f;
            for (int p = 0; p < stats_parts; ++p) {
                const float2 st = *reinterpret_cast<const float2*>(planes_lds + p * 2048 + tid * 8);
                sm += st.x;
                sq += st.y;
            }
            const float inv_k = 1.0f / (float)K;
            const float mean = sm * inv_k;
            const float var = fmaxf(fmaf(sq, inv_k, -mean * mean), 0.f);
            *reinterpret_cast<float2*>(aux + 2048 + tid * 8) = make_float2(mean, __builtin_amdgcn_rsqf(var + ln_eps));
        }
    }
    __syncthreads();   // every wave is done with the operand ring; reuse it as 8 x 16 KiB images
    char* img = smem + wid * 16384;
    if constexpr (DEEP) {   // the four 32 KiB slots other than the aux slot
        const int region = (wid >> 1) + ((wid >> 1) >= (nk % 3) ? 1 : 0);
        img = smem + region * OPERAND_BYTES + (wid & 1) * 16384;
    }
    float* prod_stats = (EPI == VPF_EPI_BIAS_RESIDUAL || EPI == VPF_EPI_PATCH) ? stats_out : nullptr;
    store_wave_tile<EPI>(img, aux, acc, wm, wn, m0, n0, lane, residual, pos, g2, C, ldc, M, N, prod_stats,
                         stats_rows);
}

}  // namespace

#define VPF_IS_LN(E) ((E) == VPF_EPI_LN || (E) == VPF_EPI_LN_GELU)
#define VPF_GEMM_LAUNCH(E)                                                                                   \
    do {                                                                                                     \
        if (kern == 2)                                                                                       \
            hipLaunchKernelGGL((k_gemm_bf16<E, false>), grid, block, 0, s, A, (int)lda, W, bias, residual, pos, \
                               patch_rows, reinterpret_cast<const float2*>(row_stats), colsum, C, (int)ldc, m, n, \
                               k, group, stats_parts, ln_eps, stats_out, stats_rows);                        \
        else if (VPF_IS_LN(E) && stats_parts > AUX_PARTS)                                                    \
            hipLaunchKernelGGL((k_gemm_bf16<E, true, VPF_IS_LN(E)>), grid, block, 0, s, A, (int)lda, W,        \
                               bias, residual, pos, patch_rows, reinterpret_cast<const float2*>(row_stats), colsum, \
                               C, (int)ldc, m, n, k, group, stats_parts, ln_eps, stats_out, stats_rows);     \
        else                                                                                                 \
            hipLaunchKernelGGL((k_gemm_bf16<E, true>), grid, block, 0, s, A, (int)lda, W, bias, residual, pos,  \
                               patch_rows, reinterpret_cast<const float2*>(row_stats), colsum, C, (int)ldc, m, n, \
                               k, group, stats_parts, ln_eps, stats_out, stats_rows);                        \
    } while (0)

static int g_group = -1;
static int tile_group() {   // VPF_GEMM_GROUP overrides the A-panel group size of the tile order (0 = tm-major)
    if (g_group < 0) { const char* e = getenv("VPF_GEMM_GROUP"); g_group = e ? atoi(e) : 4; if (g_group < 0) g_group = 0; }
    return g_group;
}

// GEMM kernel selection: 1 = k_gemm_bf16 with the deep A ring (product), 2 = the 2-stage ring (A/B timing).
// VPF_GEMM_KERNEL sets the initial value, vpf_gemm_tune() the current one.
static int g_kernel = -1;
static int gemm_kernel() {
    if (g_kernel < 0) { const char* e = getenv("VPF_GEMM_KERNEL"); g_kernel = e ? atoi(e) : 1; if (g_kernel < 1 || g_kernel > 2) g_kernel = 1; }
    return g_kernel;
}
static int tile_group();
VPF_API int vpf_gemm_tune(int kernel, int group) {
    if (kernel < 1 || kernel > 2) return VPF_ERR_ARG;
    g_kernel = kernel;
    if (group >= 0) { tile_group(); g_group = group; }
    return 0;
}

VPF_API int vpf_gemm_bf16(const uint16_t* A, int64_t lda, const uint16_t* W, const float* bias,
                          const uint16_t* residual, const float* pos, int patch_rows, const float* row_stats,
                          const float* colsum, uint16_t* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                          int epilogue, int stats_parts, float ln_eps, float* stats_out, void* stream) {
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
    if (stats_parts < 0 || stats_parts > (gemm_kernel() == 2 ? AUX_PARTS : MAX_PARTS) || !(ln_eps >= 0.f))
        return VPF_ERR_ARG;
    if (stats_out && (((uintptr_t)stats_out & 7) || (epilogue != VPF_EPI_BIAS_RESIDUAL && epilogue != VPF_EPI_PATCH)))
        return VPF_ERR_ARG;
    // producer plane stride: rows of C (EPI_PATCH interleaves one CLS row per patch_rows rows)
    const int64_t srows = epilogue == VPF_EPI_PATCH ? (M / patch_rows) * (patch_rows + 1) : M;
    if (srows > INT32_MAX) return VPF_ERR_ARG;
    const int stats_rows = (int)srows;
    const int64_t tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    if (tiles > INT32_MAX) return VPF_ERR_ARG;
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((unsigned)tiles), block(NTHREADS);
    const int kern = gemm_kernel();
    const int group = tile_group();
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
