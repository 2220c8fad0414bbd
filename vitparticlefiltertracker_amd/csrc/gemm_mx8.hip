// MX-fp8 GEMM for the fp8 weight path (BASELINE.json configs[4]; MI355X_MICROARCH.md
// "Matrix cores": block-scaled e4m3 runs at twice the bf16 MFMA rate).
//
//   C[M][N] = epi( deq(A8)[M][K] . deq(W8)[N][K]^T ),   deq(x) = e4m3(x) * 2^(e8m0 - 127) per 32 K values,
//
// on v_mfma_scale_f32_16x16x128_f8f6f4 (fp32 accumulation; the hardware applies both operands' block scales).
// Operand format (vpf.h "MX8 operands"): elements [rows][K] bytes, per 128-deep K-tile a plane of scale words
// in 64-row bricks (gemm_common.h mx8_scale_byte). Producers: vpf_quantize_mx8 (weights, CLS
// rows), and the epilogues of the residual-stream GEMMs (Out8) and of this kernel (FC1 -> FC2's A operand).
//
// Design: the bf16 kernel's geometry at twice the K per K-tile — 256x256 tile, 8 waves 2 (M) x 4 (N), each
// wave 8 x 4 fragments of 16x16 — so a K-tile is again 256 rows x 128 B per operand with the same XOR-swizzled
// lane-linear LDS image and 16-B DMA pieces, plus 1 KiB of scale words per operand (one 16-B piece per lane
// of one wave). Per K-tile a wave reads 24 ds_read_b128 (two per fragment: its 32-byte K-block) and 3 scale
// words (op_sel picks a fragment's byte), then issues 32 MFMAs (each 2x the cycles of a 16x16x32 bf16 MFMA for 4x the K). Two-stage ring
// (2 x 66 KiB) with two K-tiles of lookahead (a buffer is refilled once its K-tile sits in registers) + 28 KiB
// epilogue operands (bias | colsum | up to MX_PARTS statistics planes) = 160 KiB.
// Epilogues: gemm_common.h store_wave_tile (bias / LN fold / GELU / residual, statistics planes, optional
// MX-fp8 copy of the output).
#include "gemm_common.h"

using namespace vpf;
using namespace vpf::gemm;

typedef int i32x8 __attribute__((ext_vector_type(8)));
namespace {

constexpr int BK = 128;                                // fp8 K values per K-tile (128 B per row)
constexpr int SC_BYTES = BM * 4;                       // a K-tile's scale words for 256 rows
constexpr int STAGE = 2 * TILE_BYTES + 2 * SC_BYTES;   // A | B | A scales | B scales
constexpr int RING = 2 * STAGE;
constexpr int MX_PARTS = 13;                           // statistics planes next to bias | colsum
constexpr int AUX = 2048 + MX_PARTS * 2048;
static_assert(RING + AUX <= 160 * 1024, "LDS budget");
static_assert(8 * 16384 <= RING, "the 8 epilogue images live in the ring");

// One W fragment (column group J of the wave) against the 8 activation fragments: op_sel (an immediate)
// picks the scale byte — J of the W brick word, i % 4 of the activation brick words sa0 (i < 4) / sa1.
#define VPF_MX(I, SA) \
    acc[I] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(b, a[I], acc[I], 0, 0, J, sb, (I) & 3, SA)
template <int J>
__device__ __forceinline__ void mx_col(f32x4 (&acc)[8], const i32x8& b, const i32x8 (&a)[8], int sb, int sa0, int sa1) {
    VPF_MX(0, sa0); VPF_MX(1, sa0); VPF_MX(2, sa0); VPF_MX(3, sa0);
    VPF_MX(4, sa1); VPF_MX(5, sa1); VPF_MX(6, sa1); VPF_MX(7, sa1);
}
#undef VPF_MX
// Q8D: fp8-only LN + GELU output (FC1) stored from the accumulators (store_wave_tile_q8_direct; W rows in wperm16 order)
template <int EPI, bool OUT8, bool Q8D = false>
__global__ __launch_bounds__(NTHREADS) void k_gemm_mx8(const uint8_t* __restrict__ A, int lda,
                                                       const uint32_t* __restrict__ As, int lds_a,
                                                       const uint8_t* __restrict__ W,
                                                       const uint32_t* __restrict__ Ws,
                                                       const float* __restrict__ bias, const bf16_t* residual,
                                                       const float2* __restrict__ stats,
                                                       const float* __restrict__ colsum, bf16_t* C, int ldc,
                                                       int M, int N, int K, int group, int stats_parts,
                                                       float ln_eps, float* stats_out, Out8 o8) {
    __shared__ __attribute__((aligned(16))) char smem[RING + AUX];
    char* aux = smem + RING;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    int m0, n0;
    tile_of(M, N, group, m0, n0);

    const char* Ablk = reinterpret_cast<const char*>(A) + (size_t)m0 * lda;
    const char* Bblk = reinterpret_cast<const char*>(W) + (size_t)n0 * K;
    uint32_t offA[4], offB[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int g = i * 8 + wid;                 // wave-instruction index: rows [8g, 8g+8)
        const int row = 8 * g + (lane >> 3);
        const int lch = (lane & 7) ^ ((row >> 1) & 7);
        offA[i] = (uint32_t)min(row, M - 1 - m0) * (uint32_t)lda + (uint32_t)(lch * 16);
        offB[i] = (uint32_t)min(Q8D ? wperm16(row) : row, N - 1 - n0) * (uint32_t)K + (uint32_t)(lch * 16);
    }
    // scale words: waves 0-3 DMA the A rows' 4 x 256 B, waves 4-7 the W rows' (4 B per lane, one piece per wave,
    // so every wave issues the same 9 pieces per K-tile and the counted waits below are wave-uniform); rows past
    // the end read the last valid word (never used)
    const uint32_t* sc_src = wid < 4 ? As + min(m0 + wid * 64 + lane, lds_a - 1) : Ws + min(n0 + (wid - 4) * 64 + lane, N - 1);
    const int64_t sc_kstride = wid < 4 ? lds_a : N;
    auto stage = [&](int buf, int kt) {
        char* st = smem + buf * STAGE;
        const uint32_t koff = (uint32_t)kt * BK;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int g = i * 8 + wid;
            __builtin_amdgcn_global_load_lds((gptr_t)(Ablk + offA[i] + koff), (lptr_t)(st + g * 1024), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((gptr_t)(Bblk + offB[i] + koff), (lptr_t)(st + TILE_BYTES + g * 1024), 16,
                                             0, 0);
        }
        __builtin_amdgcn_global_load_lds((gptr_t)(sc_src + kt * sc_kstride), (lptr_t)(st + 2 * TILE_BYTES + wid * 256), 4,
                                         0, 0);
    };

    constexpr bool LN = (EPI == VPF_EPI_LN || EPI == VPF_EPI_LN_GELU);
    auto load_aux = [&]() {
        if (wid == 2)
            __builtin_amdgcn_global_load_lds((gptr_t)(bias + min(n0 + lane * 4, N - 4)), (lptr_t)aux, 16, 0, 0);
        if constexpr (LN) {
            if (wid == 3)
                __builtin_amdgcn_global_load_lds((gptr_t)(colsum + min(n0 + lane * 4, N - 4)), (lptr_t)(aux + 1024), 16,
                                                 0, 0);
            const float* sd = reinterpret_cast<const float*>(stats);
            const int planes = stats_parts > 0 ? stats_parts : 1;
            if ((M & 1) == 0 && ((uintptr_t)sd & 15) == 0) {
                for (int pc = wid; pc < 2 * planes; pc += 8) {
                    const int p = pc >> 1, hf = pc & 1;
                    __builtin_amdgcn_global_load_lds(
                        (gptr_t)(sd + (int64_t)p * 2 * M + min(2 * m0 + hf * 256 + lane * 4, 2 * M - 4)),
                        (lptr_t)(aux + 2048 + p * 2048 + hf * 1024), 16, 0, 0);
                }
            } else {
                for (int p = 0; p < planes; ++p)
                    __builtin_amdgcn_global_load_lds(
                        (gptr_t)(sd + (int64_t)p * 2 * M + min(2 * m0 + wid * 64 + lane, 2 * M - 1)),
                        (lptr_t)(aux + 2048 + p * 2048 + wid * 256), 4, 0, 0);
            }
        }
    };

    const int wm = wid >> 2, wn = wid & 3;
    const int fr = lane & 15, fq = lane >> 4;
    f32x4 acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

    // Two buffers, two K-tiles of lookahead: a K-tile's buffer is refilled as soon as every wave holds that
    // K-tile's fragments in registers (second barrier), not after its MFMAs — the DMA of K-tile t+2 flies during
    // K-tile t's MFMAs and all of K-tile t+1. Per wave, the in-flight pieces at the top of step t are K-tile
    // t+1's 9 (A 4, B 4, one scale piece): a counted vmcnt(9), never a drain inside the loop.
    const int nk = K / BK;
    // The refill is unconditional (past the end it re-reads K-tile nk-1 into the free buffer) so that it stays in
    // the MFMA basic block and its 9 DMA issues interleave with the MFMAs (sched_group_barrier below).
    load_aux();
    stage(0, 0);
    stage(1, min(1, nk - 1));
    for (int kt = 0; kt < nk; ++kt) {
        asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
        __builtin_amdgcn_s_barrier();   // K-tile kt (and the epilogue operands) landed for every wave
        asm volatile("" ::: "memory");
        const char* st = smem + (kt & 1) * STAGE;
        const char* la = st;
        const char* lb = st + TILE_BYTES;
        const uint32_t* las = reinterpret_cast<const uint32_t*>(st + 2 * TILE_BYTES);
        const uint32_t* lbs = las + BM;
        // Operand map of the 16x16x128 f8 MFMA (tools/micro/mx_probe.py, profiles/r1_gemm_lab/mx_probe.txt): lane
        // group g holds K values [16g, 16g+16) in bytes 0-15 and [64+16g, +16) in bytes 16-31 (two 16x16x64
        // halves), and the scale of K-block b = [32b, 32b+32) comes from lane group b. So a lane reads logical
        // chunks fq and 4+fq of its row, and supplies the scale of block fq: one word per 64-row brick, byte f
        // = fragment f of the brick (mx8_scale_byte).
        i32x4 bl[4], bh[4], al[8], ah[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = wn * 64 + j * 16 + fr;
            const int sw = (row >> 1) & 7;
            bl[j] = lds16(lb + row * 128 + (fq ^ sw) * 16);
            bh[j] = lds16(lb + row * 128 + ((4 + fq) ^ sw) * 16);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int row = wm * 128 + i * 16 + fr;
            const int sw = (row >> 1) & 7;
            al[i] = lds16(la + row * 128 + (fq ^ sw) * 16);
            ah[i] = lds16(la + row * 128 + ((4 + fq) ^ sw) * 16);
        }
        int sb, sa0, sa1;
        if constexpr (Q8D) {
            // LDS row j*16 + fr holds W row wperm16(j*16 + fr) = (fr >> 2)*16 + j*4 + (fr & 3) of the brick: its scale is
            // byte fr >> 2 of word j*4 + (fr & 3); the four bytes are gathered into one word (byte j) by two v_perm_b32
            const uint32_t* wb = lbs + wn * 64 + fq * 16 + (fr & 3);
            int w0 = lds4(wb), w1 = lds4(wb + 4), w2 = lds4(wb + 8), w3 = lds4(wb + 12);
            sa0 = lds4(las + (2 * wm) * 64 + fq * 16 + fr);
            sa1 = lds4(las + (2 * wm + 1) * 64 + fq * 16 + fr);
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(bl[0]), "+v"(bl[1]), "+v"(bl[2]), "+v"(bl[3]), "+v"(bh[0]), "+v"(bh[1]), "+v"(bh[2]),
                           "+v"(bh[3]), "+v"(w0), "+v"(w1), "+v"(w2), "+v"(w3), "+v"(sa0), "+v"(sa1)
                         :: "memory");
            const uint32_t f = (uint32_t)(fr >> 2);
            const uint32_t lo = __builtin_amdgcn_perm((uint32_t)w1, (uint32_t)w0, 0x0c0c0000u | ((4u + f) << 8) | f);
            const uint32_t hi = __builtin_amdgcn_perm((uint32_t)w3, (uint32_t)w2, ((4u + f) << 24) | (f << 16) | 0x0c0cu);
            sb = (int)(lo | hi);
        } else {
            sb = lds4(lbs + wn * 64 + fq * 16 + fr);
            sa0 = lds4(las + (2 * wm) * 64 + fq * 16 + fr);
            sa1 = lds4(las + (2 * wm + 1) * 64 + fq * 16 + fr);
            // the reads have landed (the wait is tied to every fragment register so no use moves above it)
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(bl[0]), "+v"(bl[1]), "+v"(bl[2]), "+v"(bl[3]), "+v"(bh[0]), "+v"(bh[1]), "+v"(bh[2]),
                           "+v"(bh[3]), "+v"(sb), "+v"(sa0), "+v"(sa1)
                         :: "memory");
        }
        asm volatile(""
                     : "+v"(al[0]), "+v"(al[1]), "+v"(al[2]), "+v"(al[3]), "+v"(al[4]), "+v"(al[5]), "+v"(al[6]),
                       "+v"(al[7]), "+v"(ah[0]), "+v"(ah[1]), "+v"(ah[2]), "+v"(ah[3]), "+v"(ah[4]), "+v"(ah[5]),
                       "+v"(ah[6]), "+v"(ah[7]));
        i32x8 a[8], b[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            b[j] = i32x8{bl[j].x, bl[j].y, bl[j].z, bl[j].w, bh[j].x, bh[j].y, bh[j].z, bh[j].w};
#pragma unroll
        for (int i = 0; i < 8; ++i)
            a[i] = i32x8{al[i].x, al[i].y, al[i].z, al[i].w, ah[i].x, ah[i].y, ah[i].z, ah[i].w};
        // the first column group's 8 MFMAs run before the buffer-release barrier (they need only registers), so the
        // MFMA pipe works while the slower waves finish their reads
        mx_col<0>(acc[0], b[0], a, sb, sa0, sa1);
        __builtin_amdgcn_s_barrier();   // every wave holds K-tile kt in registers: its buffer is free
        asm volatile("" ::: "memory");
        stage(kt & 1, min(kt + 2, nk - 1));
        // swapped operands as in the bf16 kernel: W fragment as MFMA-A, activation as MFMA-B -> D[n][m]
        mx_col<1>(acc[1], b[1], a, sb, sa0, sa1);
        mx_col<2>(acc[2], b[2], a, sb, sa0, sa1);
        mx_col<3>(acc[3], b[3], a, sb, sa0, sa1);
#pragma unroll
        for (int q = 0; q < 9; ++q) {   // one DMA issue after every 2 MFMAs
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the trailing refills land before the ring is reused

    if constexpr (LN) {
        if (stats_parts > 0 && tid < BM) {   // planes -> {mean, rstd} once per row (see gemm_bf16.hip)
            float sm = 0.f, sq = 0.f;
            for (int p = 0; p < stats_parts; ++p) {
                const float2 s2 = *reinterpret_cast<const float2*>(aux + 2048 + p * 2048 + tid * 8);
                sm += s2.x;
                sq += s2.y;
            }
            const float inv_k = 1.0f / (float)K;
            const float mean = sm * inv_k;
            const float var = fmaxf(fmaf(sq, inv_k, -mean * mean), 0.f);
            *reinterpret_cast<float2*>(aux + 2048 + tid * 8) = make_float2(mean, __builtin_amdgcn_rsqf(var + ln_eps));
        }
    }
    // no LDS-DMA is outstanding after the K loop; saying so with the builtin (which hipcc's waitcnt pass reads,
    // unlike asm) keeps it from draining vmcnt(0) - and with it the residual loads - at the first LDS access below
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    if constexpr (Q8D) {   // no LDS image: only the LN combine above needs the barrier
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        store_wave_tile_q8_direct<EPI>(aux, acc, wm, wn, m0, n0, lane, M, N, o8);
        return;
    }
    uint4 res[16];
    if constexpr (EPI == VPF_EPI_BIAS_RESIDUAL) load_residual<false>(res, residual, wm, wn, m0, n0, lane, ldc, M, N);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // raw barrier: the residual loads stay in flight
    __builtin_amdgcn_s_barrier();   // the ring is free: 8 x 16 KiB epilogue images
    asm volatile("" ::: "memory");
    float* prod_stats = EPI == VPF_EPI_BIAS_RESIDUAL ? stats_out : nullptr;
    char* img = smem + wid * 16384;
    if (OUT8 && C == nullptr) {   // fp8-only output (FC1): 16-B element stores, gathered scale words
        store_wave_tile_q8<EPI>(img, aux, acc, wm, wn, m0, n0, lane, M, N, o8);
        return;
    }
    store_wave_tile<EPI, OUT8>(img, aux, acc, wm, wn, m0, n0, lane, res, nullptr, 1, C, ldc, M, N, prod_stats, M, o8);
}

// MX quantisation of bf16 rows: one lane per 8 values, a DPP quad per 32-value block (gemm_common.h).
// Row r of X goes to row r * out_stride of X8 / the scale words (the CLS rows of a token tensor).
__global__ __launch_bounds__(256) void k_quantize_mx8(const bf16_t* __restrict__ X, int64_t ldx, int64_t rows, int K,
                                                      int64_t out_stride, uint8_t* __restrict__ X8, int64_t ld8,
                                                      uint8_t* __restrict__ S, int64_t lds) {
    const int per_row = K / 8;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = rows * per_row;
    const int64_t tc = t < total ? t : total - 1;   // whole quads are in or out (per_row % 4 == 0)
    const int64_t r = tc / per_row;
    const int c = (int)(tc - r * per_row) * 8;
    const uint4 v = *reinterpret_cast<const uint4*>(X + r * ldx + c);
    uint32_t e8;
    const uint2 q = mx8_quant8(v, e8);
    if (t < total) {
        const int64_t orow = r * out_stride;
        *reinterpret_cast<uint2*>(X8 + orow * ld8 + c) = q;
        if ((c & 31) == 0) S[mx8_scale_byte(orow, c, (int)lds)] = (uint8_t)e8;
    }
}

}  // namespace

#define VPF_MX8_ARGS                                                                                         \
    A, (int)lda, As, (int)lds_a, W, Ws, bias, residual, reinterpret_cast<const float2*>(row_stats), colsum,    \
        C, (int)ldc, (int)M, (int)N, (int)K, group, stats_parts, ln_eps, stats_out, o8
#define VPF_MX8_LAUNCH(E)                                                                                    \
    do {                                                                                                     \
        if (o8.q && !C && (E) == VPF_EPI_LN_GELU)                                                            \
            hipLaunchKernelGGL((k_gemm_mx8<E, true, (E) == VPF_EPI_LN_GELU>), grid, block, 0, s, VPF_MX8_ARGS); \
        else if (o8.q)                                                                                       \
            hipLaunchKernelGGL((k_gemm_mx8<E, true>), grid, block, 0, s, VPF_MX8_ARGS);                       \
        else                                                                                                 \
            hipLaunchKernelGGL((k_gemm_mx8<E, false>), grid, block, 0, s, VPF_MX8_ARGS);                      \
    } while (0)

VPF_API int vpf_gemm_mx8(const uint8_t* A, int64_t lda, const uint32_t* As, int64_t lds_a, const uint8_t* W,
                         const uint32_t* Ws, const float* bias, const uint16_t* residual, const float* row_stats,
                         const float* colsum, uint16_t* C, int64_t ldc, uint8_t* C8, int64_t ld8, uint32_t* Cs,
                         int64_t lds_c, int64_t M, int64_t N, int64_t K, int epilogue, int stats_parts, float ln_eps,
                         float* stats_out, void* stream) {
    if (M <= 0 || N <= 0 || K <= 0 || K % BK != 0 || N % 8 != 0 || lda < K || lda % 16 != 0) return VPF_ERR_ARG;
    if (M > INT32_MAX / 2 || N > 65536 || K > 65536 || lda > INT32_MAX / 2) return VPF_ERR_ARG;
    if ((uint64_t)BM * (uint64_t)lda > UINT32_MAX) return VPF_ERR_ARG;
    if (!A || !As || !W || !Ws || !bias || (!C && !C8)) return VPF_ERR_ARG;
    if (((uintptr_t)A & 15) || ((uintptr_t)W & 15) || ((uintptr_t)As & 15) || ((uintptr_t)Ws & 15)) return VPF_ERR_ARG;
    if (lds_a < M || lds_a % 64 != 0 || N % 64 != 0 || lds_a > INT32_MAX / 2) return VPF_ERR_ARG;
    if (C && (ldc < N || ldc % 8 != 0 || ldc > INT32_MAX / 2)) return VPF_ERR_ARG;
    if (epilogue == VPF_EPI_BIAS_RESIDUAL && (!residual || !C)) return VPF_ERR_ARG;
    const bool ln = epilogue == VPF_EPI_LN || epilogue == VPF_EPI_LN_GELU;
    if (ln && (!row_stats || !colsum)) return VPF_ERR_ARG;
    if (((uintptr_t)bias & 15) || ((uintptr_t)colsum & 15) || ((uintptr_t)row_stats & 7)) return VPF_ERR_ARG;
    if (stats_parts < 0 || stats_parts > MX_PARTS || !(ln_eps >= 0.f)) return VPF_ERR_ARG;
    if (stats_out && (((uintptr_t)stats_out & 7) || epilogue != VPF_EPI_BIAS_RESIDUAL)) return VPF_ERR_ARG;
    if (vpf_check_out8(C8, ld8, Cs, lds_c, M, N)) return VPF_ERR_ARG;
    const Out8 o8{C8, reinterpret_cast<uint8_t*>(Cs), (int)ld8, (int)lds_c};
    const int64_t tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    if (tiles > INT32_MAX) return VPF_ERR_ARG;
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((unsigned)tiles), block(NTHREADS);
    const int group = vpf_gemm_tile_group_mx8(epilogue);
    switch (epilogue) {
        case VPF_EPI_BIAS: VPF_MX8_LAUNCH(VPF_EPI_BIAS); break;
        case VPF_EPI_BIAS_GELU: VPF_MX8_LAUNCH(VPF_EPI_BIAS_GELU); break;
        case VPF_EPI_BIAS_RESIDUAL: VPF_MX8_LAUNCH(VPF_EPI_BIAS_RESIDUAL); break;
        case VPF_EPI_LN: VPF_MX8_LAUNCH(VPF_EPI_LN); break;
        case VPF_EPI_LN_GELU: VPF_MX8_LAUNCH(VPF_EPI_LN_GELU); break;
        default: return VPF_ERR_ARG;   // EPI_PATCH: the patch embedding stays bf16 (K = 3 p^2, 0.7 % of FLOPs)
    }
    VPF_RETURN_LAUNCH();
}

VPF_API int vpf_quantize_mx8(const uint16_t* X, int64_t ldx, int64_t rows, int64_t K, int64_t out_stride,
                             uint8_t* X8, int64_t ld8, uint32_t* S, int64_t lds, void* stream) {
    if (rows <= 0 || K <= 0 || K % 128 != 0 || ldx < K || ldx % 8 != 0 || out_stride < 1) return VPF_ERR_ARG;
    if (!X || !X8 || !S || ((uintptr_t)X & 15) || ((uintptr_t)X8 & 7) || ((uintptr_t)S & 3)) return VPF_ERR_ARG;
    if (ld8 < K || ld8 % 8 != 0 || lds < (rows - 1) * out_stride + 1 || lds % 64 != 0 || lds > INT32_MAX / 4)
        return VPF_ERR_ARG;
    const int64_t total = rows * (K / 8);
    const int64_t blocks = (total + 255) / 256;
    if (blocks > INT32_MAX || K > 65536) return VPF_ERR_ARG;
    hipLaunchKernelGGL(k_quantize_mx8, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const bf16_t*>(X), ldx, rows, (int)K, out_stride, X8, ld8,
                       reinterpret_cast<uint8_t*>(S), lds);
    VPF_RETURN_LAUNCH();
}
