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
//    the refills are issued from the MFMA block: B(t+1)'s DMA right behind the fragment reads, A(t+2)'s four
//    issues interleaved into the 64 MFMAs per wave (one per 16), instead of 8 back-to-back issues after the
//    barrier while the MFMA pipes idle (QKV / proj / FC1 / FC2 -1.8..-4.5 %, profiles/r1_gemm_lab/ilv_ab.txt).
//  * MFMA operands are "swapped" (W fragment as A, activation fragment as B) so the accumulator holds
//    D[n][m]: each lane owns 4 consecutive output columns of one row. Epilogue (gemm_common.h): bias
//    (+ GELU, gelu_sig2) in fp32 on the accumulators, bf16 pack, 8-B writes into a per-wave XOR-swizzled
//    LDS image, then fully coalesced 16-B row stores (+ 16-B residual reads / position-embedding adds), and
//    optionally an MX-fp8 copy of the output (the A operand of the MX8 GEMMs, gemm_mx8.hip).
//  * Workgroup -> tile mapping is XCD-aware (bijective remap, cdna_hip_programming.md §5 T1): the blocks
//    that share an XCD walk consecutive tiles of one 256-row A panel, so the panel is an L2 hit.
#include <algorithm>
#include "gemm_common.h"

using namespace vpf;
using namespace vpf::gemm;

namespace {

constexpr int BK = 64;
constexpr int OPERAND_BYTES = BM * BK * 2;      // 32 KiB per operand tile
static_assert(OPERAND_BYTES == TILE_BYTES, "bf16 K-tile geometry");
// epilogue operands: bias (1 KiB) | colsum (1 KiB) | row statistics (up to AUX_PARTS planes of 2 KiB).
// 16 planes (D = 1024) do not fit next to bias / colsum: the deep ring then lands them in a second free A
// slot at the last K-step (wide path).
constexpr int AUX_PARTS = 15;
constexpr int MAX_PARTS = 16;
constexpr int AUX_BYTES = 2048 + AUX_PARTS * 2048;

// WIDE: LN-folded consumers of more than AUX_PARTS statistics planes (ViT-L: 16); the planes land in the second free
// A slot at the last K-step. OUT8: residual-stream producers that also write an MX-fp8 copy of their output.
// PART (vpf_gemm_bf16_splitk): blockIdx.y = split s of gridDim.y; the block runs K-tiles [s K/S, (s+1) K/S) and stores
// its raw fp32 accumulators to the partial plane s ((float*)C + s M N, row-major [M][N]) with no epilogue.
template <int EPI, bool WIDE = false, bool OUT8 = false, bool PART = false>
__global__ __launch_bounds__(NTHREADS) void k_gemm_bf16(const bf16_t* __restrict__ A, int lda,
                                                        const bf16_t* __restrict__ W,
                                                        const float* __restrict__ bias,
                                                        const bf16_t* residual,
                                                        const float* __restrict__ pos, int g2,
                                                        const float2* __restrict__ stats,
                                                        const float* __restrict__ colsum,
                                                        bf16_t* C, int ldc, int M, int N, int K, int group,
                                                        int stats_parts, float ln_eps, float* stats_out,
                                                        int stats_rows, Out8 o8) {
    // Deep ring: A ring of 3 K-tiles (A prefetched 2 K-tiles ahead: the activation panel is the operand that misses
    // L2), B ring of 2 (weights stay L2-hot); 5 x 32 KiB = all 160 KiB of LDS, and the epilogue operands go into the
    // A slot no K-tile uses any more (slot nk % 3, DMA'd at K-tile max(nk-2, 0)).
    constexpr int SMEM = 5 * OPERAND_BYTES;
    static_assert(AUX_BYTES <= OPERAND_BYTES, "aux region must fit the free A slot of the deep ring");
    __shared__ __attribute__((aligned(16))) char smem[SMEM];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);

    int m0, n0;
    tile_of(M, N, group, m0, n0);   // XCD-aware grouped tile order (gemm_common.h)
    // the GELU epilogues store straight from the accumulators (store_wave_tile_direct: W rows permuted in the DMA)
    constexpr bool DIRECT = (EPI == VPF_EPI_LN_GELU || EPI == VPF_EPI_BIAS_GELU) && !OUT8 && !PART;

    // ---- per-lane DMA source offsets (bytes, relative to the block's panel base) ----
    const int kbase = PART ? (int)blockIdx.y * (K / (int)gridDim.y) : 0;   // PART: this split's first K column
    const char* Ablk = reinterpret_cast<const char*>(A) + (size_t)m0 * lda * 2 + (size_t)kbase * 2;
    const char* Bblk = reinterpret_cast<const char*>(W) + (size_t)n0 * K * 2 + (size_t)kbase * 2;
    uint32_t offA[4], offB[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int g = i * 8 + wid;                 // wave-instruction index: rows [8g, 8g+8)
        const int row = 8 * g + (lane >> 3);
        const int pch = lane & 7;
        const int lch = pch ^ ((row >> 1) & 7);    // logical chunk stored at this physical slot
        const int ra = min(row, M - 1 - m0);
        const int rb = min(DIRECT ? wperm(row) : row, N - 1 - n0);
        offA[i] = (uint32_t)ra * (uint32_t)(lda * 2) + (uint32_t)(lch * 16);
        offB[i] = (uint32_t)rb * (uint32_t)(K * 2) + (uint32_t)(lch * 16);
    }
    auto stage_a = [&](int kt) {   // A K-tile kt -> A slot kt % 3
        char* la = smem + (kt % 3) * OPERAND_BYTES;
        const uint32_t koff = (uint32_t)kt * (BK * 2);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds((gptr_t)(Ablk + offA[i] + koff), (lptr_t)(la + (i * 8 + wid) * 1024), 16, 0, 0);
    };
    auto stage_b = [&](int kt) {   // B K-tile kt -> B slot kt & 1
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

    // Epilogue operands ride the DMA stream into the aux region of LDS (bias | colsum | per-row (mean, rstd)), so their
    // latency hides under the K loop and nothing epilogue-related stays live in VGPRs across it (holding them in
    // registers cost ~10 % on the LayerNorm-folded GEMMs: 250 VGPRs). Out-of-range columns / rows read clamped (valid)
    // addresses; their values are never stored.
    constexpr bool LN = (EPI == VPF_EPI_LN || EPI == VPF_EPI_LN_GELU) && !PART;
    const int nk = (PART ? K / (int)gridDim.y : K) / BK;
    char* aux = smem + (nk % 3) * OPERAND_BYTES;
    // stats_parts == 0: one {mean, rstd} plane; else stats_parts {sum, sumsq} planes of M rows each. A plane's 256-row
    // slice is 2 KiB = two 16-B-per-lane pieces (M even, 16-B aligned base), dealt round-robin over the 8 waves (12
    // planes: 3 pieces per wave instead of 12 4-B pieces).
    constexpr bool wide = LN && WIDE;   // host: only for stats_parts > AUX_PARTS
    char* planes_lds = wide ? smem + ((nk + 1) % 3) * OPERAND_BYTES : aux + 2048;
    // The epilogue-operand DMAs re-read the lane id (opaque_lane): their per-lane addresses are then computed where they
    // are issued (once per tile) instead of being hoisted above the K loop, where they would stay live across it.
    auto load_planes = [&](char* dst) {
        const int lane = opaque_lane();
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
        if constexpr (PART) return;   // no epilogue operands
        const int lane = opaque_lane();
        if (wid == 0)
            __builtin_amdgcn_global_load_lds((gptr_t)(bias + min(n0 + lane * 4, N - 4)), (lptr_t)aux, 16, 0, 0);
        if constexpr (LN) {
            if (wid == 1)
                __builtin_amdgcn_global_load_lds((gptr_t)(colsum + min(n0 + lane * 4, N - 4)), (lptr_t)(aux + 1024), 16,
                                                 0, 0);
            if (!wide) load_planes(aux + 2048);
        }
    };
    stage_a(0);
    stage_b(0);
    if (nk > 1) stage_a(1);
    // The epilogue operands must land before a barrier that every wave passes ahead of the epilogue: one wave DMAs the
    // bias, others the colsum and the planes, and every wave reads all of them. At nk >= 2 they are issued at K-tile
    // nk - 2 and the last K-step's vmcnt(0) + barrier retires them; at nk == 1 (K = 64) that barrier is the loop's only
    // one, so they go out with the prologue (issued after it, the direct-store GELU epilogue read bias that
    // waves 0 / 1 had not yet landed).
    if (nk == 1) load_aux();
    for (int kt = 0; kt < nk; ++kt) {
        // issue order: A0 B0 A1 | per K-tile t: B(t+1) A(t+2). A(kt), B(kt) are older than everything but A(kt+1)
        // (4 pieces per wave) until the last two K-tiles, where the tail is B / aux only.
        if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (nk >= 2 && kt == nk - 2) load_aux();
        if (wide && kt == nk - 1) load_planes(planes_lds);   // slot of A(nk-2): free after this barrier
        const char* la = smem + (kt % 3) * OPERAND_BYTES;
        const char* lb = smem + (3 + (kt & 1)) * OPERAND_BYTES;
        // both 32-deep halves' fragments are read up front (24 ds_read_b128): the second half's reads complete under
        // the first half's 32 MFMAs instead of stalling between them
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
        // The refills are issued from the MFMA block, after the fragment reads in program order (a DMA into LDS is never
        // hoisted over an LDS read; MFMAs may pass it): B(t+1)'s 4 issues right behind the reads, whose latency they
        // overlap, then A(t+2)'s 4 interleaved one per 16 MFMAs, instead of 8 back-to-back issues after the barrier
        // while the MFMA pipes idle (QKV / proj / FC1 / FC2 -1.8..-4.5 %, profiles/r1_gemm_lab/ilv_ab.txt).
        // Unconditional, so they stay in this block: past the end they re-read K-tile nk-1 into that K-tile's own slot
        // (identical bytes). Program order B, A keeps the counted vmcnt(4) at the next barrier meaning "B(t+1) has
        // landed".
        stage_b(min(kt + 1, nk - 1));
        stage_a(min(kt + 2, nk - 1));
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[ks][j], a[ks][i], acc[j][i], 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 24, 0);   // the 24 fragment reads
        __builtin_amdgcn_sched_group_barrier(0x020, 4, 0);    // B(t+1)'s DMA
#pragma unroll
        for (int q = 0; q < 4; ++q) {                          // 16 MFMAs per A(t+2) DMA issue
            __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
    }

    if constexpr (PART) {
        __builtin_amdgcn_s_waitcnt(0x0F70);   // the past-the-end refills land before the wave exits
        // lane: output row m0 + wm*128 + i*16 + (lane & 15), columns n0 + wn*64 + j*16 + 4*(lane >> 4) .. +3
        float* P = reinterpret_cast<float*>(C) + (size_t)blockIdx.y * M * N;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int m = m0 + wm * 128 + i * 16 + fr;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int n = n0 + wn * 64 + j * 16 + fq * 4;
                if (m < M && n < N) *reinterpret_cast<f32x4*>(P + (size_t)m * N + n) = acc[j][i];
            }
        }
        return;
    }
    // ---------------- epilogue ----------------
    if constexpr (LN) {
        // statistics planes -> {mean, rstd} once per row (in place over plane 0, which only this thread reads), instead
        // of in each of the 4 waves that share the row; the aux DMA landed before the last K-step's barrier
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
    // no LDS-DMA is outstanding after the K loop; saying so with the builtin (which hipcc's waitcnt pass reads, unlike
    // asm) keeps it from draining vmcnt(0) - and with it the residual loads - at the first LDS access below
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    uint4 res[16];
    constexpr bool PIPE = EPI != VPF_EPI_PATCH && !OUT8;
    if constexpr (DIRECT) {
        if constexpr (LN) {   // the LN combine above is read by the other waves
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
        store_wave_tile_direct<EPI>(aux, acc, wm, wn, m0, n0, lane, C, ldc, M, N);
        return;
    }
    if constexpr (EPI == VPF_EPI_BIAS_RESIDUAL) load_residual<PIPE>(res, residual, wm, wn, m0, n0, lane, ldc, M, N);
    // every wave is done with the operand ring (reused as 8 x 16 KiB images) and the LN combine is visible; a raw
    // barrier, so the residual loads stay in flight across it (no DMA is outstanding after the K loop)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // the four 32 KiB slots other than the aux slot
    const int region = (wid >> 1) + ((wid >> 1) >= (nk % 3) ? 1 : 0);
    char* img = smem + region * OPERAND_BYTES + (wid & 1) * 16384;
    if constexpr (PIPE) {
        store_wave_tile_pipe<EPI>(img, aux, acc, wm, wn, m0, n0, lane, res, C, ldc, M, N,
                                  EPI == VPF_EPI_BIAS_RESIDUAL ? stats_out : nullptr, stats_rows);
    } else {
        float* prod_stats = (EPI == VPF_EPI_BIAS_RESIDUAL || EPI == VPF_EPI_PATCH) ? stats_out : nullptr;
        store_wave_tile<EPI, OUT8>(img, aux, acc, wm, wn, m0, n0, lane, res, pos, g2, C, ldc, M, N, prod_stats,
                                   stats_rows, o8);
    }
}

// ---------------------------------------------------------------------------------------------------------------
// Ping-pong main loop (cdna_hip_programming.md §5 "The 256² 8-phase template", T3+T4): same tile, waves and
// epilogues as k_gemm_bf16, different sync structure.
//  * A K-tile is cut into four 16 KiB half-tiles, one per quadrant operand of a wave's 128x64 sub-tile:
//    A0 / A1 = the A rows of quadrant-row mh = 0 / 1 of BOTH wave rows (rows g*128 + mh*64 + r), B0 / B1 = the
//    W rows of quadrant-column nh = 0 / 1 of all four wave columns (rows wn*64 + nh*32 + r). Slot (buffer, type)
//    = 16 KiB at ((kt & 1) * 4 + type) * 16 KiB; 128 KiB ring + 32 KiB epilogue operands.
//  * Four phases per K-tile, one output quadrant (16 MFMAs) each: q0 (mh0,nh0) reads A0 + B0, q1 (mh0,nh1)
//    reads B1, q2 (mh1,nh1) reads A1, q3 (mh1,nh0) reads nothing (A1, B0 still in registers). Phase body:
//    [fragment reads | one half-tile DMA (2 pieces per wave) | counted vmcnt] barrier [lgkmcnt(0), 16 MFMAs]
//    barrier.
//  * The wave row wm = 1 runs one barrier behind wm = 0 (one extra barrier before the loop, matched by wm = 0
//    after it): the two waves that share a SIMD alternate, one issuing MFMAs while the other issues its LDS
//    reads and DMA (ping-pong).
//  * Half-tiles are consumed in the order n = 4k + {A0, B0, B1, A1} and half-tile n is DMA'd in phase n - 6:
//    q0 of K-tile t stages B1(t+1), q1 A1(t+1), q2 A0(t+2), q3 B0(t+2). WAR: a slot is re-staged >= 2 phases
//    after the phase that last read it (the reads of both wave rows are retired by then). RAW: the vmcnt(8) at
//    the end of the memory part of phase p leaves the 4 youngest half-tiles (n = p+3 .. p+6) in flight and
//    retires n <= p+2, which phase p+1 reads after one more barrier. q2 needs no wait (q3 reads nothing).
//  * Past the last K-tile the DMAs re-stage K-tile nk-1 (identical bytes), so every phase is branch-free.
template <int EPI, bool OUT8 = false>
__global__ __launch_bounds__(NTHREADS) void k_gemm_pp(const bf16_t* __restrict__ A, int lda,
                                                      const bf16_t* __restrict__ W,
                                                      const float* __restrict__ bias,
                                                      const bf16_t* residual,
                                                      const float* __restrict__ pos, int g2,
                                                      const float2* __restrict__ stats,
                                                      const float* __restrict__ colsum,
                                                      bf16_t* C, int ldc, int M, int N, int K, int group,
                                                      int stats_parts, float ln_eps, float* stats_out,
                                                      int stats_rows, Out8 o8) {
    constexpr int HALF = 16384;
    constexpr int RING = 8 * HALF;   // 2 buffers x {A0, B0, B1, A1}
    static_assert(RING + AUX_BYTES <= 160 * 1024, "LDS budget");
    __shared__ __attribute__((aligned(16))) char smem[RING + AUX_BYTES];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid >> 2, wn = wid & 3;

    int m0, n0;
    tile_of(M, N, group, m0, n0);
    constexpr bool DIRECT = (EPI == VPF_EPI_LN_GELU || EPI == VPF_EPI_BIAS_GELU) && !OUT8;

    const char* Ablk = reinterpret_cast<const char*>(A) + (size_t)m0 * lda * 2;
    const char* Bblk = reinterpret_cast<const char*>(W) + (size_t)n0 * K * 2;
    // per-lane DMA source offsets: [type][piece]; piece p of a half-tile = local rows (wid + 8p) * 8 + lane / 8
    uint32_t off[4][2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int rho = (wid + 8 * p) * 8 + (lane >> 3);             // local row 0..127
        const int lch = (lane & 7) ^ ((rho >> 1) & 7);               // logical chunk at this physical slot
        const int ra0 = (rho >> 6) * 128 + (rho & 63);               // A0: g*128 + r
        const int rb0 = (rho >> 5) * 64 + (DIRECT ? wperm(rho & 31) : (rho & 31));   // B0: wn*64 + r
        const int ra[2] = {ra0, ra0 + 64}, rb[2] = {rb0, rb0 + 32};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            off[h == 0 ? 0 : 3][p] = (uint32_t)min(ra[h], M - 1 - m0) * (uint32_t)(lda * 2) + (uint32_t)(lch * 16);
            off[h == 0 ? 1 : 2][p] = (uint32_t)min(rb[h], N - 1 - n0) * (uint32_t)(K * 2) + (uint32_t)(lch * 16);
        }
    }
    const int nk = K / BK;
    // type: 0 = A0, 1 = B0, 2 = B1, 3 = A1
    auto stage = [&](int type, int kt) {
        kt = min(kt, nk - 1);
        char* slot = smem + ((kt & 1) * 4 + type) * HALF;
        const char* src = (type == 0 || type == 3) ? Ablk : Bblk;
        const uint32_t koff = (uint32_t)kt * (BK * 2);
#pragma unroll
        for (int p = 0; p < 2; ++p)
            __builtin_amdgcn_global_load_lds((gptr_t)(src + off[type][p] + koff), (lptr_t)(slot + (wid + 8 * p) * 1024),
                                             16, 0, 0);
    };

    // epilogue operands (same layout as k_gemm_bf16's aux region), issued first: retired by the prologue wait
    constexpr bool LN = (EPI == VPF_EPI_LN || EPI == VPF_EPI_LN_GELU);
    char* aux = smem + RING;
    if (wid == 0)
        __builtin_amdgcn_global_load_lds((gptr_t)(bias + min(n0 + lane * 4, N - 4)), (lptr_t)aux, 16, 0, 0);
    if constexpr (LN) {
        if (wid == 1)
            __builtin_amdgcn_global_load_lds((gptr_t)(colsum + min(n0 + lane * 4, N - 4)), (lptr_t)(aux + 1024), 16, 0, 0);
        const float* sd = reinterpret_cast<const float*>(stats);
        const int planes = stats_parts > 0 ? stats_parts : 1;
        if ((M & 1) == 0 && ((uintptr_t)sd & 15) == 0) {
            for (int pc = wid; pc < 2 * planes; pc += 8) {
                const int p = pc >> 1, hf = pc & 1;
                __builtin_amdgcn_global_load_lds((gptr_t)(sd + (int64_t)p * 2 * M + min(2 * m0 + hf * 256 + lane * 4, 2 * M - 4)),
                                                 (lptr_t)(aux + 2048 + p * 2048 + hf * 1024), 16, 0, 0);
            }
        } else {
            for (int p = 0; p < planes; ++p)
                __builtin_amdgcn_global_load_lds((gptr_t)(sd + (int64_t)p * 2 * M + min(2 * m0 + wid * 64 + lane, 2 * M - 1)),
                                                 (lptr_t)(aux + 2048 + p * 2048 + wid * 256), 4, 0, 0);
        }
    }
    // prologue: half-tiles n = 0..5 (K-tile 0 whole, A0 / B0 of K-tile 1); retire n <= 1 (+ the aux pieces)
    stage(0, 0); stage(1, 0); stage(2, 0); stage(3, 0); stage(0, 1); stage(1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (wm == 1) __builtin_amdgcn_s_barrier();   // the ping-pong offset
    asm volatile("" ::: "memory");

    f32x4 acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int fr = lane & 15, fq = lane >> 4;
    // fragment read byte offsets inside a half-tile slot (without the k-chunk term): A rows wm*64 + i*16 + fr,
    // B rows wn*32 + j*16 + fr; (row >> 1) & 7 = (fr >> 1) & 7 for every fragment (row bases are multiples of 16)
    const int sw = (fr >> 1) & 7;
    const int abase = (wm * 64 + fr) * 128, bbase = (wn * 32 + fr) * 128;
    auto mfma_quadrant = [&](const i32x4 (&fa)[2][4], const i32x4 (&fb)[2][2], int mh, int nh) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    acc[nh * 2 + j][mh * 4 + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        __builtin_bit_cast(bf16x8, fb[ks][j]), __builtin_bit_cast(bf16x8, fa[ks][i]),
                        acc[nh * 2 + j][mh * 4 + i], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto read_a = [&](i32x4 (&fa)[2][4], const char* slot) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i) fa[ks][i] = lds16(slot + abase + i * 2048 + (((ks * 4 + fq) ^ sw) << 4));
    };
    auto read_b = [&](i32x4 (&fb)[2][2], const char* slot) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int j = 0; j < 2; ++j) fb[ks][j] = lds16(slot + bbase + j * 2048 + (((ks * 4 + fq) ^ sw) << 4));
    };
    auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };

    for (int kt = 0; kt < nk; ++kt) {
        const char* buf = smem + (kt & 1) * 4 * HALF;
        i32x4 fa0[2][4], fa1[2][4], fb0[2][2], fb1[2][2];
        // q0: (mh0, nh0)
        read_a(fa0, buf);
        read_b(fb0, buf + HALF);
        stage(2, kt + 1);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        bar();
        mfma_quadrant(fa0, fb0, 0, 0);
        bar();
        // q1: (mh0, nh1)
        read_b(fb1, buf + 2 * HALF);
        stage(3, kt + 1);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        bar();
        mfma_quadrant(fa0, fb1, 0, 1);
        bar();
        // q2: (mh1, nh1)
        read_a(fa1, buf + 3 * HALF);
        stage(0, kt + 2);
        bar();
        mfma_quadrant(fa1, fb1, 1, 1);
        bar();
        // q3: (mh1, nh0)
        stage(1, kt + 2);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        bar();
        mfma_quadrant(fa1, fb0, 1, 0);
        bar();
    }
    if (wm == 0) __builtin_amdgcn_s_barrier();   // matches wm = 1's offset barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the clamped re-stages past the end

    // ---------------- epilogue (k_gemm_bf16's, on the ring's 8 x 16 KiB) ----------------
    if constexpr (LN) {
        if (stats_parts > 0 && tid < BM) {
            float sm = 0.f, sq = 0.f;
            for (int p = 0; p < stats_parts; ++p) {
                const float2 st = *reinterpret_cast<const float2*>(aux + 2048 + p * 2048 + tid * 8);
                sm += st.x;
                sq += st.y;
            }
            const float inv_k = 1.0f / (float)K;
            const float mean = sm * inv_k;
            const float var = fmaxf(fmaf(sq, inv_k, -mean * mean), 0.f);
            *reinterpret_cast<float2*>(aux + 2048 + tid * 8) = make_float2(mean, __builtin_amdgcn_rsqf(var + ln_eps));
        }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): nothing outstanding (see k_gemm_bf16)
    uint4 res[16];
    constexpr bool PIPE = EPI != VPF_EPI_PATCH && !OUT8;
    if constexpr (DIRECT) {
        if constexpr (LN) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
        store_wave_tile_direct<EPI>(aux, acc, wm, wn, m0, n0, lane, C, ldc, M, N);
        return;
    }
    if constexpr (EPI == VPF_EPI_BIAS_RESIDUAL) load_residual<PIPE>(res, residual, wm, wn, m0, n0, lane, ldc, M, N);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    char* img = smem + wid * 16384;
    if constexpr (PIPE) {
        store_wave_tile_pipe<EPI>(img, aux, acc, wm, wn, m0, n0, lane, res, C, ldc, M, N,
                                  EPI == VPF_EPI_BIAS_RESIDUAL ? stats_out : nullptr, stats_rows);
    } else {
        float* prod_stats = (EPI == VPF_EPI_BIAS_RESIDUAL || EPI == VPF_EPI_PATCH) ? stats_out : nullptr;
        store_wave_tile<EPI, OUT8>(img, aux, acc, wm, wn, m0, n0, lane, res, pos, g2, C, ldc, M, N, prod_stats,
                                   stats_rows, o8);
    }
}

}  // namespace

#define VPF_IS_LN(E) ((E) == VPF_EPI_LN || (E) == VPF_EPI_LN_GELU)
#define VPF_IS_PROD(E) ((E) == VPF_EPI_BIAS_RESIDUAL || (E) == VPF_EPI_PATCH)
#define VPF_GEMM_ARGS                                                                                        \
    A, (int)lda, W, bias, residual, pos, patch_rows, reinterpret_cast<const float2*>(row_stats), colsum, C,     \
        (int)ldc, m, n, k, group, stats_parts, ln_eps, stats_out, stats_rows, o8
// fp8 copies are produced by the residual-stream producers only (proj, patch embed): the only bf16 GEMMs whose output
// an MX8 GEMM reads. Kernel 5 (the ping-pong loop) holds at most AUX_PARTS planes next to its ring.
#define VPF_GEMM_LAUNCH(E)                                                                                   \
    do {                                                                                                     \
        if (kern == 5 && !(VPF_IS_LN(E) && stats_parts > AUX_PARTS) && o8.q == nullptr)                      \
            hipLaunchKernelGGL((k_gemm_pp<E, false>), grid, block, 0, s, VPF_GEMM_ARGS);                     \
        else if (kern == 5 && VPF_IS_PROD(E) && o8.q != nullptr)                                             \
            hipLaunchKernelGGL((k_gemm_pp<E, VPF_IS_PROD(E)>), grid, block, 0, s, VPF_GEMM_ARGS);            \
        else if (VPF_IS_LN(E) && stats_parts > AUX_PARTS)                                                    \
            hipLaunchKernelGGL((k_gemm_bf16<E, VPF_IS_LN(E)>), grid, block, 0, s, VPF_GEMM_ARGS);             \
        else if (VPF_IS_PROD(E) && o8.q != nullptr)                                                          \
            hipLaunchKernelGGL((k_gemm_bf16<E, false, VPF_IS_PROD(E)>), grid, block, 0, s, VPF_GEMM_ARGS);    \
        else                                                                                                 \
            hipLaunchKernelGGL((k_gemm_bf16<E>), grid, block, 0, s, VPF_GEMM_ARGS);                           \
    } while (0)

// Kernel and tile order per shape. The product library has two bf16 kernels, bit-identical on every output
// (test_gemm_kernel_variants_bit_identical): 1 = k_gemm_bf16 (deep ring, refills from the MFMA block), 5 = the ping-pong
// loop k_gemm_pp. The A/B variants of earlier rounds (2-stage ring, refills after the barrier, two-pass epilogue, the
// four-wave AGPR loop, staggered starts, the persistent kernel, the mid-K barrier loop, timing probes) live in the lab
// build (tools/gemm_lab, libvpf_lab.so); no environment variable selects a kernel here.
//  * QKV (the LN-folded bias-only epilogue) runs kernel 5: 2.5 % faster there in one process (2.603 vs 2.670 ms,
//    profiles/r2_gemm_lab/kernel_ab_r2s5.txt). FC1 (LN + GELU) runs kernel 5 since its epilogue stores straight from
//    the accumulators (store_wave_tile_direct): 3.751 vs 3.817 ms (profiles/r4_lab/fc1_direct_kernel_group_ab.txt);
//    with the LDS-image epilogue the two kernels were level on FC1. Every other epilogue is fastest on kernel 1.
//  * Tile order (A panels per group; the order never changes a bit), profiles/r2_gemm_lab/group_sweep_r2.txt: the
//    N <= 1024 GEMMs (proj / FC2: 3 column tiles) are 1-1.5 % faster with 2 panels per group (FC2 3.196 vs 3.226 ms,
//    proj 1.070 vs 1.082), QKV with 4; FC1 (LN + GELU, 12 column tiles at ViT-B) takes 8: 16 was -0.9 % on FC1 and
//    -0.7 % on the frame against 4 (fc1_group16_pmc.txt), and 8 another 0.3-0.5 % ahead of 16 (group_sweep_r2s5.txt,
//    fc1_pp_group_ab.txt).
// vpf_gemm_tune(kernel, group) is an explicit test / A/B hook: kernel 1 or 5 for every shape (and a fixed group when
// group >= 0), 0 = back to the per-shape defaults. It is process state set by a call, never read from the environment.
constexpr int kDefaultGroup = 4;
static int g_kernel = 0;   // 0: per-shape default; 1 / 5: forced by vpf_gemm_tune
static int g_group = -1;   // -1: per-shape default
static int gemm_kernel_for(int epilogue) {
    if (g_kernel) return g_kernel;
    return (epilogue == VPF_EPI_LN || epilogue == VPF_EPI_LN_GELU) ? 5 : 1;
}
static int tile_group_for(int64_t N, int epilogue) {
    if (g_group >= 0) return g_group;
    if (N <= 1024) return 2;
    return epilogue == VPF_EPI_LN_GELU ? 8 : kDefaultGroup;
}
int vpf_gemm_tile_group() { return g_group >= 0 ? g_group : kDefaultGroup; }   // shared with gemm_mx8.hip
// MX8 GEMMs' default group (profiles/r2_gemm_lab/mx8_group_sweep.txt, fp8 frames): the LN-folded bias-only QKV is ~5 %
// faster with 8 A panels per group (1.93-1.95 vs 2.05 ms); proj / FC1 / FC2 keep 4.
int vpf_gemm_tile_group_mx8(int epilogue) {
    if (g_group >= 0) return g_group;
    return epilogue == VPF_EPI_LN ? 8 : kDefaultGroup;
}
VPF_API int vpf_gemm_tune(int kernel, int group) {
    if (kernel != 0 && kernel != 1 && kernel != 5) return VPF_ERR_ARG;
    if (group < -1 || group > 64) return VPF_ERR_ARG;
    g_kernel = kernel;
    g_group = kernel == 0 ? -1 : group;
    return 0;
}

// fp8 output operand check shared with gemm_mx8.hip: element rows ld8 >= N bytes (8-B aligned pieces), scale
// planes of lds_c >= output rows words (lds_c % 64 == 0, mx8_scale_byte), N % 128 == 0.
int vpf_check_out8(const uint8_t* C8, int64_t ld8, const uint32_t* Cs, int64_t lds_c, int64_t rows, int64_t N) {
    if (!C8) return Cs ? VPF_ERR_ARG : 0;
    if (!Cs || N % 128 != 0 || ld8 < N || ld8 % 8 != 0 || ((uintptr_t)C8 & 7) || lds_c < rows || lds_c % 64 != 0 ||
        ((uintptr_t)Cs & 3) || ld8 > INT32_MAX || lds_c > INT32_MAX / 4)
        return VPF_ERR_ARG;
    return 0;
}

VPF_API int vpf_gemm_bf16(const uint16_t* A, int64_t lda, const uint16_t* W, const float* bias,
                          const uint16_t* residual, const float* pos, int patch_rows, const float* row_stats,
                          const float* colsum, uint16_t* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                          int epilogue, int stats_parts, float ln_eps, float* stats_out, uint8_t* C8, int64_t ld8,
                          uint32_t* Cs, int64_t lds_c, void* stream) {
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
    if (stats_parts < 0 || stats_parts > MAX_PARTS || !(ln_eps >= 0.f))
        return VPF_ERR_ARG;
    if (stats_out && (((uintptr_t)stats_out & 7) || (epilogue != VPF_EPI_BIAS_RESIDUAL && epilogue != VPF_EPI_PATCH)))
        return VPF_ERR_ARG;
    // producer plane stride: rows of C (EPI_PATCH interleaves one CLS row per patch_rows rows)
    const int64_t srows = epilogue == VPF_EPI_PATCH ? (M / patch_rows) * (patch_rows + 1) : M;
    if (srows > INT32_MAX) return VPF_ERR_ARG;
    const int stats_rows = (int)srows;
    // fp8 copy of C: residual-stream producers only, deep-ring kernel
    if (C8 && epilogue != VPF_EPI_BIAS_RESIDUAL && epilogue != VPF_EPI_PATCH) return VPF_ERR_ARG;
    if (vpf_check_out8(C8, ld8, Cs, lds_c, srows, N)) return VPF_ERR_ARG;
    const Out8 o8{C8, reinterpret_cast<uint8_t*>(Cs), (int)ld8, (int)lds_c};
    const int64_t tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    if (tiles > INT32_MAX) return VPF_ERR_ARG;
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((unsigned)tiles), block(NTHREADS);
    const int kern = gemm_kernel_for(epilogue);
    const int group = tile_group_for(N, epilogue);
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

// ---------------------------------------------------------------------------------------------------------------
// Split-K form for GEMMs with few rows (the last block's CLS-row GEMMs: M = particles per GPU, so 6 - 48 output
// tiles each running the whole K loop on one CU). S blocks per tile each run K/S (k_gemm_bf16<PART>) into fp32
// partial planes; k_splitk_reduce sums the S planes in split order (fixed: the result does not depend on M) and
// applies the epilogue with the semantics of vpf_gemm_bf16's: LN / LN_GELU from {mean, rstd} row statistics,
// BIAS / BIAS_GELU, BIAS_RESIDUAL (bf16(acc + b) + residual, rounded again) with optional statistics planes of the
// stored values. One thread per 8 consecutive columns of a row; a 64-column plane block is 8 lanes (xor shuffles).
template <int EPI>
__global__ __launch_bounds__(256) void k_splitk_reduce(const float* __restrict__ P, int S, int M, int N,
                                                       const float* __restrict__ bias,
                                                       const float2* __restrict__ stats,
                                                       const float* __restrict__ colsum, const bf16_t* residual,
                                                       bf16_t* C, int64_t ldc, float* stats_out) {
    constexpr bool LN = (EPI == VPF_EPI_LN || EPI == VPF_EPI_LN_GELU);
    constexpr bool GELU = (EPI == VPF_EPI_BIAS_GELU || EPI == VPF_EPI_LN_GELU);
    const int per_row = N >> 3;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = t < (int64_t)M * per_row;
    const int m = live ? (int)(t / per_row) : 0;
    const int n = live ? (int)(t - (int64_t)m * per_row) * 8 : 0;
    float v[8];
    if (live) {
        const float* p = P + (size_t)m * N + n;
        const float4 a0 = *reinterpret_cast<const float4*>(p), a1 = *reinterpret_cast<const float4*>(p + 4);
        v[0] = a0.x; v[1] = a0.y; v[2] = a0.z; v[3] = a0.w; v[4] = a1.x; v[5] = a1.y; v[6] = a1.z; v[7] = a1.w;
        for (int s = 1; s < S; ++s) {
            const float* q = p + (size_t)s * M * N;
            const float4 b0 = *reinterpret_cast<const float4*>(q), b1 = *reinterpret_cast<const float4*>(q + 4);
            v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w; v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
        }
        float rstd = 1.f, nrm = 0.f;
        if constexpr (LN) {
            const float2 st = stats[m];
            rstd = st.y;
            nrm = -st.y * st.x;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            float y = LN ? fmaf(rstd, v[e], fmaf(nrm, colsum[n + e], bias[n + e])) : v[e] + bias[n + e];
            if constexpr (GELU) {
                const f32x2 g = gelu_sig2(f32x2{y, y});
                y = g.x;
            }
            v[e] = y;
        }
    }
    uint32_t o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = pack_bf2(v[2 * e], v[2 * e + 1]);
    if constexpr (EPI == VPF_EPI_BIAS_RESIDUAL) {
        if (live) {
            const uint4 rv = *reinterpret_cast<const uint4*>(residual + (size_t)m * ldc + n);
            const uint32_t rr[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
                o[e] = pack_bf2(bf2f((bf16_t)(o[e] & 0xffff)) + bf2f((bf16_t)(rr[e] & 0xffff)),
                                bf2f((bf16_t)(o[e] >> 16)) + bf2f((bf16_t)(rr[e] >> 16)));
        }
        if (stats_out != nullptr) {   // {sum, sumsq} of the stored values over this lane's 64-column block
            float s1 = 0.f, s2 = 0.f;
            if (live) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float lo = bf2f((bf16_t)(o[e] & 0xffff)), hi = bf2f((bf16_t)(o[e] >> 16));
                    s1 += lo + hi;
                    s2 = fmaf(lo, lo, s2);
                    s2 = fmaf(hi, hi, s2);
                }
            }
#pragma unroll
            for (int x = 1; x < 8; x <<= 1) {
                s1 += __shfl_xor(s1, x, 64);
                s2 += __shfl_xor(s2, x, 64);
            }
            if (live && (n & 63) == 0)
                *reinterpret_cast<float2*>(stats_out + ((int64_t)(n >> 6) * M + m) * 2) = make_float2(s1, s2);
        }
    }
    if (live) *reinterpret_cast<uint4*>(C + (size_t)m * ldc + n) = make_uint4(o[0], o[1], o[2], o[3]);
}

VPF_API int vpf_gemm_bf16_splitk(const uint16_t* A, int64_t lda, const uint16_t* W, const float* bias,
                                 const uint16_t* residual, const float* row_stats, const float* colsum, uint16_t* C,
                                 int64_t ldc, int64_t M, int64_t N, int64_t K, int epilogue, int splits,
                                 float* stats_out, float* partial_ws, int64_t ws_elems, void* stream) {
    if (M <= 0 || N <= 0 || K <= 0 || splits < 1 || K % ((int64_t)splits * BK) != 0 || N % 8 != 0 || lda < K ||
        lda % 8 != 0 || ldc < N || ldc % 8 != 0)
        return VPF_ERR_ARG;
    if (M > INT32_MAX / 2 || N > 65536 || K > 65536 || lda > INT32_MAX / 2 || ldc > INT32_MAX / 2 || splits > 64)
        return VPF_ERR_ARG;
    if ((uint64_t)BM * (uint64_t)lda * 2 > UINT32_MAX) return VPF_ERR_ARG;
    if (!A || !W || !bias || !C || !partial_ws || ws_elems < (int64_t)splits * M * N) return VPF_ERR_ARG;
    if (((uintptr_t)partial_ws & 15) || ((uintptr_t)C & 15) || ((uintptr_t)A & 15) || ((uintptr_t)W & 15))
        return VPF_ERR_ARG;
    const bool ln = epilogue == VPF_EPI_LN || epilogue == VPF_EPI_LN_GELU;
    if (ln && (!row_stats || !colsum || ((uintptr_t)row_stats & 7))) return VPF_ERR_ARG;
    if (epilogue == VPF_EPI_BIAS_RESIDUAL && (!residual || ((uintptr_t)residual & 15))) return VPF_ERR_ARG;
    if (stats_out && (epilogue != VPF_EPI_BIAS_RESIDUAL || N % 64 != 0 || ((uintptr_t)stats_out & 7)))
        return VPF_ERR_ARG;
    if (epilogue != VPF_EPI_BIAS && epilogue != VPF_EPI_BIAS_GELU && epilogue != VPF_EPI_BIAS_RESIDUAL && !ln)
        return VPF_ERR_ARG;
    const int64_t tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    if (tiles > 65535 * 256) return VPF_ERR_ARG;
    hipStream_t s = (hipStream_t)stream;
    const int m = (int)M, n = (int)N, k = (int)K;
    const Out8 o8{nullptr, nullptr, 0, 0};
    hipLaunchKernelGGL((k_gemm_bf16<VPF_EPI_BIAS, false, false, true>),
                       dim3((unsigned)tiles, (unsigned)splits), dim3(NTHREADS), 0, s, reinterpret_cast<const bf16_t*>(A),
                       (int)lda, reinterpret_cast<const bf16_t*>(W), nullptr, nullptr, nullptr, 1, nullptr, nullptr,
                       reinterpret_cast<bf16_t*>(partial_ws), n, m, n, k, vpf_gemm_tile_group(), 0, 0.f, nullptr, m, o8);
    const int e = (int)hipGetLastError();
    if (e) return e;
    const int64_t threads = M * (N / 8);
    const dim3 rg((unsigned)((threads + 255) / 256));
    const float2* st = reinterpret_cast<const float2*>(row_stats);
    const bf16_t* R = reinterpret_cast<const bf16_t*>(residual);
    bf16_t* Cb = reinterpret_cast<bf16_t*>(C);
    switch (epilogue) {
        case VPF_EPI_BIAS:
            hipLaunchKernelGGL(k_splitk_reduce<VPF_EPI_BIAS>, rg, dim3(256), 0, s, partial_ws, splits, m, n, bias, st,
                               colsum, R, Cb, ldc, nullptr);
            break;
        case VPF_EPI_BIAS_GELU:
            hipLaunchKernelGGL(k_splitk_reduce<VPF_EPI_BIAS_GELU>, rg, dim3(256), 0, s, partial_ws, splits, m, n, bias,
                               st, colsum, R, Cb, ldc, nullptr);
            break;
        case VPF_EPI_BIAS_RESIDUAL:
            hipLaunchKernelGGL(k_splitk_reduce<VPF_EPI_BIAS_RESIDUAL>, rg, dim3(256), 0, s, partial_ws, splits, m, n,
                               bias, st, colsum, R, Cb, ldc, stats_out);
            break;
        case VPF_EPI_LN:
            hipLaunchKernelGGL(k_splitk_reduce<VPF_EPI_LN>, rg, dim3(256), 0, s, partial_ws, splits, m, n, bias, st,
                               colsum, R, Cb, ldc, nullptr);
            break;
        default:
            hipLaunchKernelGGL(k_splitk_reduce<VPF_EPI_LN_GELU>, rg, dim3(256), 0, s, partial_ws, splits, m, n, bias,
                               st, colsum, R, Cb, ldc, nullptr);
            break;
    }
    VPF_RETURN_LAUNCH();
}
