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
#include <stdlib.h>
#include <algorithm>
#include <type_traits>
#include "gemm_common.h"

using namespace vpf;
using namespace vpf::gemm;

namespace {

constexpr int BK = 64;
#ifndef VPF_ILV_SPACING
#define VPF_ILV_SPACING 16   // MFMAs per A(t+2) DMA issue in the product loop; -D builds A/B variants (tools/ab_libs.sh)
#endif
constexpr int OPERAND_BYTES = BM * BK * 2;      // 32 KiB per operand tile
static_assert(OPERAND_BYTES == TILE_BYTES, "bf16 K-tile geometry");
constexpr int STAGE_BYTES = 2 * OPERAND_BYTES;  // A + B
constexpr int LDS_BYTES = 2 * STAGE_BYTES;      // 128 KiB
// epilogue operands: bias (1 KiB) | colsum (1 KiB) | row statistics (up to AUX_PARTS planes of 2 KiB).
// 16 planes (D = 1024) do not fit next to bias / colsum: the deep ring then lands them in a second free A
// slot at the last K-step (wide path).
constexpr int AUX_PARTS = 15;
constexpr int MAX_PARTS = 16;
constexpr int AUX_BYTES = 2048 + AUX_PARTS * 2048;

// LAB (A/B timing only, vpf_gemm_tune kernels 8 - 12): 1 = the C stores predicated off at run time (all epilogue
// math, image traffic and residual loads kept), 2 = no epilogue at all (the accumulators kept alive by an empty asm),
// 3 = kernel 1 with a staggered start: the first workgroup on each CU sleeps phase x nk x ~1000 cycles, phase =
// (block >> 3) mod 2^(group >> 17), so the CUs' epilogue store bursts fall in different phases of the tile period.
// PART (vpf_gemm_bf16_splitk): blockIdx.y = split s of gridDim.y; the block runs K-tiles [s K/S, (s+1) K/S) and stores
// its raw fp32 accumulators to the partial plane s ((float*)C + s M N, row-major [M][N]) with no epilogue.
template <int EPI, bool DEEP, bool WIDE = false, bool OUT8 = false, bool ILV = true, bool PIPED_EPI = true,
          bool PAR = true, int LAB = 0, bool PART = false, bool MID = false>
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
    static_assert(!MID || (DEEP && ILV && !PART && LAB == 0), "MID: the deep-ring product kernel's loop only");
    // DEEP: A ring of 3 K-tiles (A prefetched 2 K-tiles ahead: the activation panel is the operand that
    // misses L2), B ring of 2 (weights stay L2-hot); 5 x 32 KiB = all 160 KiB of LDS, and the epilogue
    // operands go into the A slot no K-tile uses any more (slot nk % 3, DMA'd at K-tile max(nk-2, 0)).
    // !DEEP: the 2-stage A+B ring (2 x 64 KiB + 4 KiB aux), kept for A/B timing (vpf_gemm_tune).
    constexpr int SMEM = DEEP ? 5 * OPERAND_BYTES : LDS_BYTES + AUX_BYTES;
    static_assert(AUX_BYTES <= OPERAND_BYTES, "aux region must fit the free A slot of the deep ring");
    __shared__ __attribute__((aligned(16))) char smem[SMEM];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);

    int m0, n0;
    tile_of(M, N, LAB ? (group & 0xffff) : group, m0, n0);   // XCD-aware grouped tile order (gemm_common.h)
    if constexpr (LAB == 3) {   // ~T / nph per phase, T ~ nk x 4600 cycles (one K-tile ~2.3 us incl. the fixed cost)
        const int lg = group >> 17;
        if ((int)blockIdx.x < 256) {
            const int steps = (((int)blockIdx.x >> 3) & ((1 << lg) - 1)) * (K / 64);
            for (int i = 0; i < steps; ++i) {
                if (lg == 1) __builtin_amdgcn_s_sleep(36);
                else if (lg == 2) __builtin_amdgcn_s_sleep(18);
                else __builtin_amdgcn_s_sleep(9);
            }
        }
    }

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
    // LAB 4: the operand DMAs through per-panel buffer resources (k_gemm_pt's form: one tile-independent VGPR offset per
    // operand, rows past M / N read 0 and are never stored)
    const __amdgpu_buffer_rsrc_t rsA =
        __builtin_amdgcn_make_buffer_rsrc((void*)(A + (size_t)m0 * lda), (short)0, min(M - m0, BM) * lda * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsB =
        __builtin_amdgcn_make_buffer_rsrc((void*)(W + (size_t)n0 * K), (short)0, min(N - n0, BN) * K * 2, 0x00020000);
    uint32_t voffA = 0, voffB = 0;
    // LAB 5 - 8 (lab kernels 20 - 23): cache-policy bits on the K-loop DMAs (A nt / A sc0 / B nt / A sc1)
    constexpr int AUXA = LAB == 5 ? 2 : LAB == 6 ? 1 : LAB == 8 ? 16 : 0;
    constexpr int AUXB = LAB == 7 ? 2 : 0;
    if constexpr (LAB == 4) {
        const int row = 8 * wid + (lane >> 3);
        const int lch = (lane & 7) ^ ((row >> 1) & 7);
        voffA = (uint32_t)row * (uint32_t)(lda * 2) + (uint32_t)(lch * 16);
        voffB = (uint32_t)row * (uint32_t)(K * 2) + (uint32_t)(lch * 16);
    }
    auto stage_a = [&](int kt) {   // DEEP: A K-tile kt -> A slot kt % 3
        char* la = smem + (kt % 3) * OPERAND_BYTES;
        const uint32_t koff = (uint32_t)kt * (BK * 2);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if constexpr (LAB == 4)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lptr_t)(la + (i * 8 + wid) * 1024), 16, voffA,
                                                         i * 64 * lda * 2 + (int)koff, 0, 0);
            else
                __builtin_amdgcn_global_load_lds((gptr_t)(Ablk + offA[i] + koff), (lptr_t)(la + (i * 8 + wid) * 1024), 16, 0, AUXA);
        }
    };
    auto stage_b = [&](int kt) {   // DEEP: B K-tile kt -> B slot kt & 1
        char* lb = smem + (3 + (kt & 1)) * OPERAND_BYTES;
        const uint32_t koff = (uint32_t)kt * (BK * 2);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if constexpr (LAB == 4)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lptr_t)(lb + (i * 8 + wid) * 1024), 16, voffB,
                                                         i * 64 * K * 2 + (int)koff, 0, 0);
            else
                __builtin_amdgcn_global_load_lds((gptr_t)(Bblk + offB[i] + koff), (lptr_t)(lb + (i * 8 + wid) * 1024), 16, 0, AUXB);
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
    constexpr bool LN = (EPI == VPF_EPI_LN || EPI == VPF_EPI_LN_GELU) && !PART;
    const int nk = (PART ? K / (int)gridDim.y : K) / BK;
    char* aux = DEEP ? smem + (nk % 3) * OPERAND_BYTES : smem + LDS_BYTES;
    // stats_parts == 0: one {mean, rstd} plane; else stats_parts {sum, sumsq} planes of M rows each. A
    // plane's 256-row slice is 2 KiB = two 16-B-per-lane pieces (M even, 16-B aligned base), dealt round-robin
    // over the 8 waves (12 planes: 3 pieces per wave instead of 12 4-B pieces).
    constexpr bool wide = DEEP && LN && WIDE;   // host: only for stats_parts > AUX_PARTS
    char* planes_lds = wide ? smem + ((nk + 1) % 3) * OPERAND_BYTES : aux + 2048;
    // The epilogue-operand DMAs re-read the lane id (opaque_lane): their per-lane addresses are then computed where they
    // are issued (once per tile) instead of being hoisted above the K loop, where MID's register pressure spilled them
    // and the reload's vmcnt(0) drained the in-flight refills.
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
    if constexpr (!DEEP) {
        load_aux();
        stage(0, 0);
    } else {
        stage_a(0);
        stage_b(0);
        if (nk > 1) stage_a(1);
    }
    if constexpr (MID) {
        // MID: the K-tile's barrier sits between its two 32-deep halves' MFMA blocks, so every fragment read overlaps
        // MFMAs that do not wait for it. Per K-tile kt (Bar(kt) = the barrier after which tile kt is readable and every
        // read of tile kt-1 has completed):
        //   Bar(kt) -> refills B(kt+1), A(kt+2) (the slots of tile kt-1: as kernel 1) -> reads R(kt, ks 0) into F0,
        //   under MFMA(kt-1, ks 1) on F1 -> wait F0 -> reads R(kt, ks 1) into F1, under MFMA(kt, ks 0) on F0 ->
        //   wait F1 (every read of tile kt done) -> counted vmcnt + Bar(kt+1) while MFMA(kt, ks 0) drains.
        // The per-accumulator MFMA order (kt, then ks) is kernel 1's: outputs are bit-identical. Fragment reads are
        // inline asm (lds16), waited by an lgkmcnt(0) statement naming every destination: hipcc would otherwise put a
        // vmcnt(0) drain of the in-flight refills in front of reads issued after them.
        i32x4 fa[2][8], fb[2][4];
        auto read_half = [&](const char* la_, const char* lb_, int ks) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int row = wn * 64 + j * 16 + fr;
                fb[ks][j] = lds16(lb_ + row * 128 + (((ks * 4 + fq) ^ ((row >> 1) & 7)) * 16));
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int row = wm * 128 + i * 16 + fr;
                fa[ks][i] = lds16(la_ + row * 128 + (((ks * 4 + fq) ^ ((row >> 1) & 7)) * 16));
            }
        };
        auto wait_half = [&](int ks) {
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(fa[ks][0]), "+v"(fa[ks][1]), "+v"(fa[ks][2]), "+v"(fa[ks][3]), "+v"(fa[ks][4]),
                           "+v"(fa[ks][5]), "+v"(fa[ks][6]), "+v"(fa[ks][7]), "+v"(fb[ks][0]), "+v"(fb[ks][1]),
                           "+v"(fb[ks][2]), "+v"(fb[ks][3])
                         :: "memory");
        };
        auto mfma_half = [&](int ks) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fb[ks][j]),
                                                                        __builtin_bit_cast(bf16x8, fa[ks][i]), acc[j][i],
                                                                        0, 0, 0);
        };
        auto slot_a = [&](int kt) { return (const char*)smem + (kt % 3) * OPERAND_BYTES; };
        auto slot_b = [&](int kt) { return (const char*)smem + (3 + (kt & 1)) * OPERAND_BYTES; };
        // Bar(0): A0, B0 landed (A1 may stay in flight)
        if (nk > 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        auto iter = [&](int kt, auto first_) {
            // (after Bar(kt)) the epilogue operands into the A slot no K-tile uses any more, as kernel 1
            if (kt == (nk >= 2 ? nk - 2 : 0)) load_aux();
            if (wide && kt == nk - 1) load_planes(planes_lds);
            read_half(slot_a(kt), slot_b(kt), 0);
            __builtin_amdgcn_sched_barrier(0);
            // refills: B(kt+1) -> the B slot of tile kt-1, A(kt+2) -> its A slot (past the end: the last K-tile into
            // its own slot, identical bytes), one per 4 MFMAs of MFMA(kt-1, ks 1); program order B, A keeps the
            // counted vmcnt(4) at Bar(kt+1) meaning "B(kt+1) and A(kt+1) have landed"
            stage_b(min(kt + 1, nk - 1));
            stage_a(min(kt + 2, nk - 1));
            if constexpr (!decltype(first_)::value) {
                mfma_half(1);
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            wait_half(0);
            read_half(slot_a(kt), slot_b(kt), 1);
            __builtin_amdgcn_sched_barrier(0);
            mfma_half(0);
            __builtin_amdgcn_sched_barrier(0);
            wait_half(1);                                          // every read of tile kt done
            if (kt + 1 < nk) {
                if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();                      // Bar(kt+1)
                asm volatile("" ::: "memory");
            }
        };
        iter(0, std::true_type{});
        for (int kt = 1; kt < nk; ++kt) iter(kt, std::false_type{});
        mfma_half(1);                                              // MFMA(nk-1, ks 1)
    }
    // LAB 12 (lab kernel 27): an L2 prefetch D = (group >> 17) K-tiles ahead of the DMA stream. At the end of K-step kt
    // waves 0-3 touch one 128-B line of each of A's 256 rows of K-tile kt + D, waves 4-7 W's (one global_load_dword
    // per lane into a register nothing reads, kept live to the post-loop vmcnt(0)), so the later LDS-DMA of that
    // K-tile finds it in L2. The touch is the youngest memory op of its K-step, so the next barrier's counted wait
    // becomes vmcnt(5).
    constexpr bool PFE = LAB == 12;
    const int pfd = PFE ? ((group >> 17) & 15) : 0;
    int pfreg = 0;
    const char* pfbase = nullptr;
    if constexpr (PFE) {
        const int r = 64 * (wid & 3) + lane;
        pfbase = wid < 4 ? Ablk + (size_t)min(r, M - 1 - m0) * lda * 2 : Bblk + (size_t)min(r, N - 1 - n0) * K * 2;
    }
    for (int kt = 0; kt < (MID ? 0 : nk); ++kt) {
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
            if (kt + 1 < nk) {
                if (PFE && kt >= 1 && kt - 1 + pfd < nk) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            // LAB 13 (lab kernel 29, round 4): the K loop without its per-K-step barrier (each wave waits only for its own
            // DMA pieces, then reads the tile whatever the other waves' pieces hold): a timing bound on what any
            // wave-decoupled handshake could gain over the barrier; outputs are garbage
            if constexpr (LAB != 13) __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if (!ILV && kt + 1 < nk) stage_b(kt + 1);
            if (!ILV && kt + 2 < nk) stage_a(kt + 2);
            if (kt == (nk >= 2 ? nk - 2 : 0)) load_aux();
            if (wide && kt == nk - 1) load_planes(planes_lds);   // slot of A(nk-2): free after this barrier
            la = smem + (kt % 3) * OPERAND_BYTES;
            lb = smem + (3 + (kt & 1)) * OPERAND_BYTES;
        }
        // both 32-deep halves' fragments are read up front (24 ds_read_b128): the second half's reads
        // complete under the first half's 32 MFMAs instead of stalling between them
        bf16x8 a[2][8], b[2][4];
        // LAB 9 / 10 / 11 (lab kernels 24 / 25 / 26, no epilogue): the K loop with only its DMAs / DMAs + fragment reads /
        // DMAs + MFMAs on register-resident fragments, to split the loop's time between the three pipes
        constexpr bool READS = !(LAB == 9 || LAB == 11), MFMAS = !(LAB == 9 || LAB == 10);
        if constexpr (READS) {
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
        } else {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
                for (int j = 0; j < 4; ++j) b[ks][j] = bf16x8{(short)(fr + j), 1, 2, 3, 4, 5, 6, (short)ks};
#pragma unroll
                for (int i = 0; i < 8; ++i) a[ks][i] = bf16x8{(short)(fq + i), 1, 2, 3, 4, 5, 6, (short)ks};
            }
        }
        // ILV: the refills are issued from the MFMA block, after the fragment reads in program order (a DMA into
        // LDS is never hoisted over an LDS read; MFMAs may pass it): B(t+1)'s 4 issues right behind the reads,
        // whose latency they overlap, then A(t+2)'s 4 interleaved one per 16 MFMAs, instead of 8 back-to-back
        // issues after the barrier while the MFMA pipes idle. Unconditional, so they stay in this block: past
        // the end they re-read K-tile nk-1 into that K-tile's own slot (identical bytes). Program order B, A
        // keeps the counted vmcnt(4) at the next barrier meaning "B(t+1) has landed".
        // LAB 14 / 15 / 16 (lab kernels 30 / 31 / 32, round 4, no epilogue): the K loop with the B refills / the A
        // refills / all refills skipped after the prologue (reads and MFMAs on stale slots, garbage outputs): how much
        // of the loop the operand DMA bytes cost (a 256 x 384 tile would cut DMA bytes per FLOP by 17 %)
        if constexpr (DEEP && ILV) {
            if constexpr (LAB != 14 && LAB != 16) stage_b(min(kt + 1, nk - 1));
            if constexpr (LAB != 15 && LAB != 16) stage_a(min(kt + 2, nk - 1));
        }
        if constexpr (MFMAS) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[ks][j], a[ks][i], acc[j][i], 0, 0, 0);
        } else if constexpr (READS) {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
                for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(b[ks][j]));
#pragma unroll
                for (int i = 0; i < 8; ++i) asm volatile("" ::"v"(a[ks][i]));
            }
        }
        if constexpr (LAB >= 9 && LAB <= 11) {
        } else if constexpr (DEEP && ILV) {
            __builtin_amdgcn_sched_group_barrier(0x100, 24, 0);   // the 24 fragment reads
            __builtin_amdgcn_sched_group_barrier(0x020, 4, 0);    // B(t+1)'s DMA
#pragma unroll
            for (int q = 0; q < 4; ++q) {                          // VPF_ILV_SPACING MFMAs per A(t+2) DMA issue
                __builtin_amdgcn_sched_group_barrier(0x008, VPF_ILV_SPACING, 0);
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            }
            if constexpr (VPF_ILV_SPACING < 16) __builtin_amdgcn_sched_group_barrier(0x008, 64 - 4 * VPF_ILV_SPACING, 0);
        } else {
            __builtin_amdgcn_sched_group_barrier(0x100, 24, 0);   // the 24 fragment reads first
            __builtin_amdgcn_sched_group_barrier(0x008, 64, 0);   // then the 64 MFMAs (counted lgkmcnt waits)
        }
        if constexpr (PFE) {
            if (kt + pfd < nk) {
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("global_load_dword %0, %1, off" : "+v"(pfreg) : "v"(pfbase + (uint32_t)(kt + pfd) * 128)
                             : "memory");
            }
        }
    }
    if constexpr (PFE) {   // the touches' destination stays reserved until every touch has landed
        __builtin_amdgcn_s_waitcnt(0x0F70);
        asm volatile("" ::"v"(pfreg));
    }

    if constexpr (PART) {
        __builtin_amdgcn_s_waitcnt(0x0F70);   // the past-the-end refills land before the wave exits
        // lane: output row m0 + wm*128 + i*16 + (lane & 15), columns n0 + wn*64 + j*16 + 4*(lane >> 4) .. +3
        float* P = reinterpret_cast<float*>(C) + (size_t)blockIdx.y * M * N;
        const int fr = lane & 15, fq = lane >> 4;
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
    if constexpr (LAB == 2 || (LAB >= 9 && LAB <= 11) || (LAB >= 14 && LAB <= 16)) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < 8; ++i) asm volatile("" ::"v"(acc[j][i]));
        __builtin_amdgcn_s_waitcnt(0x0F70);
        return;
    }
    if constexpr (LAB == 1) { if (group & 0x10000) C = nullptr; }
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
    // no LDS-DMA is outstanding after the K loop; saying so with the builtin (which hipcc's waitcnt pass reads,
    // unlike asm) keeps it from draining vmcnt(0) - and with it the residual loads - at the first LDS access below
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    uint4 res[16];
    constexpr bool PIPE = PIPED_EPI && EPI != VPF_EPI_PATCH && !OUT8;
    if constexpr (EPI == VPF_EPI_BIAS_RESIDUAL) load_residual<PIPE && PAR>(res, residual, wm, wn, m0, n0, lane, ldc, M, N);
    // every wave is done with the operand ring (reused as 8 x 16 KiB images) and the LN combine is visible; a
    // raw barrier, so the residual loads stay in flight across it (no DMA is outstanding after the K loop)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    char* img = smem + wid * 16384;
    if constexpr (DEEP) {   // the four 32 KiB slots other than the aux slot
        const int region = (wid >> 1) + ((wid >> 1) >= (nk % 3) ? 1 : 0);
        img = smem + region * OPERAND_BYTES + (wid & 1) * 16384;
    }
    if constexpr (PIPE) {
        store_wave_tile_pipe<EPI, PAR, LAB == 1>(img, aux, acc, wm, wn, m0, n0, lane, res, C, ldc, M, N,
                                                 EPI == VPF_EPI_BIAS_RESIDUAL ? stats_out : nullptr, stats_rows);
    } else {
        float* prod_stats = (EPI == VPF_EPI_BIAS_RESIDUAL || EPI == VPF_EPI_PATCH) ? stats_out : nullptr;
        store_wave_tile<EPI, OUT8>(img, aux, acc, wm, wn, m0, n0, lane, res, pos, g2, C, ldc, M, N, prod_stats,
                                   stats_rows, o8);
    }
}

// ---------------------------------------------------------------------------------------------------------------
// Persistent form of k_gemm_bf16 for the epilogues without a residual (QKV: LN, FC1: LN + GELU; BIAS, BIAS_GELU).
// Measured on kernel 1 (vpf_gemm_tune 8 / 9, profiles/r2_gemm_lab/nostore_ab.txt): its C stores cost QKV 0.29 ms and
// FC1 0.45 ms per launch (11 %) although they are pipelined with the epilogue math: a workgroup ends only once its
// stores have completed, and the next one on that CU starts with an empty operand ring. A staggered start of the
// CUs did not change that (stagger_ab.txt), so the fix is to overlap the stores with the next tile's main loop:
//  * one workgroup per CU; block b (XCD b & 7) walks its XCD's range of logical tiles with stride gridDim / 8, in the
//    same grouped order as kernel 1;
//  * the operand stream runs on across tiles: the ring position of K-tile 0 advances by nk + 1 per tile (A slot
//    (G + kt) % 3, B slot 3 + (G + kt) & 1; the skipped A position is the epilogue-operand slot). The last K-step
//    (peeled) DMAs the next tile's A0 into the A slot of K-tile nk - 2; after the epilogue barrier its B0 and A1 go
//    into the slots of K-tile nk - 1, then the epilogue runs on a 2 KiB-per-wave image (one 16-row group at a time,
//    store_wave_tile_pipe<IMG16>) in the remaining B slot, and its 16 stores per wave stay in flight into the next
//    tile's first K-step: that step waits vmcnt(20) (A1 + the stores outstanding), a full tile's store count being
//    fixed; after an edge tile it waits vmcnt(4). gfx950 has one vmcnt for loads and stores, so the second K-step's
//    wait includes the stores: they have the epilogue tail and one K-step to drain.
//  * Outputs are bit-identical to kernel 1 (same MFMA order, same epilogue math).
// MODE (A/B): 0 = the next tile's first K-step waits vmcnt(4) (the stores included); 1 = vmcnt(20) (A1 and the 16
// stores outstanding); 2 = B1 is also DMA'd before the epilogue (the image moves to the upper half of the epilogue-
// operand slot, free once the LN combine has run), so the next tile's first two K-steps wait past the stores.
template <int EPI, int MODE = 1>
__global__ __launch_bounds__(NTHREADS) void k_gemm_pt(const bf16_t* __restrict__ A, int lda, const bf16_t* __restrict__ W,
                                                      const float* __restrict__ bias, const float2* __restrict__ stats,
                                                      const float* __restrict__ colsum, bf16_t* C, int ldc, int M, int N,
                                                      int K, int group, int stats_parts, float ln_eps) {
    static_assert(EPI == VPF_EPI_LN || EPI == VPF_EPI_LN_GELU || EPI == VPF_EPI_BIAS || EPI == VPF_EPI_BIAS_GELU,
                  "residual / patch epilogues use k_gemm_bf16");
    constexpr bool LN = (EPI == VPF_EPI_LN || EPI == VPF_EPI_LN_GELU);
    __shared__ __attribute__((aligned(16))) char smem[5 * OPERAND_BYTES];
    const int wid = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    // The lane id is re-read (opaque asm) at the top of every tile and again before its epilogue, so the per-lane
    // address math of the K loop and of the epilogue is recomputed where it is used instead of being hoisted out of
    // the tile loop, where it would stay live across the K loop (~70 spilled VGPRs, whose reloads drain vmcnt).
    int lane = opaque_lane();
    const int wm = wid >> 2, wn = wid & 3;
    const int nk = K / BK;
    const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    const int xcd = blockIdx.x & 7, stride = gridDim.x >> 3;
    const int lid_end = xcd_first(tiles, xcd + 1);
    int lid = xcd_first(tiles, xcd) + (blockIdx.x >> 3);
    if (lid >= lid_end) return;
    int m0, n0;
    tile_of_lid(M, N, group, lid, m0, n0);

    // Operand DMA through buffer resources (buffer_load ... lds): one per operand panel of the current tile (A: of the
    // next one from the last K-step on), with the panel's valid rows as the range, so rows past M / N read 0
    // (never stored) instead of clamped addresses, and the per-lane offset is tile-independent: piece i of a K-tile
    // = rows 64 i + 8 wid + lane / 8, the same swizzled chunk for every i; the row and K offsets go in soffset.
    __amdgpu_buffer_rsrc_t rsA, rsB;
    auto setup_a = [&](int tm0) {
        rsA = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (size_t)tm0 * lda), (short)0, min(M - tm0, BM) * lda * 2,
                                                0x00020000);
    };
    auto setup_b = [&](int tn0) {
        rsB = __builtin_amdgcn_make_buffer_rsrc((void*)(W + (size_t)tn0 * K), (short)0, min(N - tn0, BN) * K * 2,
                                                0x00020000);
    };
    uint32_t voffA, voffB;
    {
        const int row = 8 * wid + (lane >> 3);
        const int lch = (lane & 7) ^ ((row >> 1) & 7);
        voffA = (uint32_t)row * (uint32_t)(lda * 2) + (uint32_t)(lch * 16);
        voffB = (uint32_t)row * (uint32_t)(K * 2) + (uint32_t)(lch * 16);
    }
    auto stage_a = [&](int pos, int kt) {   // A K-tile kt -> A slot pos % 3
        char* la = smem + (pos % 3) * OPERAND_BYTES;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lptr_t)(la + (i * 8 + wid) * 1024), 16, voffA,
                                                     i * 64 * lda * 2 + kt * (BK * 2), 0, 0);
    };
    auto stage_b = [&](int pos, int kt) {   // B K-tile kt -> B slot pos & 1
        char* lb = smem + (3 + (pos & 1)) * OPERAND_BYTES;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lptr_t)(lb + (i * 8 + wid) * 1024), 16, voffB,
                                                     i * 64 * K * 2 + kt * (BK * 2), 0, 0);
    };
    // The same DMAs as inline asm for the ones issued at the tile boundary (the next tile's A0, B0, A1): hipcc's
    // waitcnt pass does not see them, so it does not drain them with a vmcnt(0) before the epilogue's LDS accesses;
    // the K loop's counted waits and barriers order them (below).
    auto dma_asm = [&](__amdgpu_buffer_rsrc_t rs, char* slot, uint32_t voff, int soff_base, int row_step) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t l = (uint32_t)(size_t)(lptr_t)(slot + (i * 8 + wid) * 1024);
            // M0 is compiler-reserved: set, used and restored inside the statement, with the M0 -> LDS-DMA wait
            // state and the SALU-written-descriptor pad (cdna_hip_programming.md §5.7)
            uint32_t keep;
            asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
                         "buffer_load_dwordx4 %1, %2, %3 offen lds\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep)
                         : "v"(voff), "s"(rs), "s"(soff_base + i * row_step), "s"(l)
                         : "memory");
        }
    };
    auto stage_a_asm = [&](int pos, int kt) {
        dma_asm(rsA, smem + (pos % 3) * OPERAND_BYTES, voffA, kt * (BK * 2), 64 * lda * 2);
    };
    auto stage_b_asm = [&](int pos, int kt) {
        dma_asm(rsB, smem + (3 + (pos & 1)) * OPERAND_BYTES, voffB, kt * (BK * 2), 64 * K * 2);
    };
    auto read_frags = [&](const char* la, const char* lb, bf16x8 (&a)[2][8], bf16x8 (&b)[2][4], int lane) {
        const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int row = wn * 64 + j * 16 + fr;
                b[ks][j] = *reinterpret_cast<const bf16x8*>(lb + row * 128 + (((ks * 4 + fq) ^ ((row >> 1) & 7)) * 16));
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int row = wm * 128 + i * 16 + fr;
                a[ks][i] = *reinterpret_cast<const bf16x8*>(la + row * 128 + (((ks * 4 + fq) ^ ((row >> 1) & 7)) * 16));
            }
        }
    };

    setup_a(m0);
    setup_b(n0);
    int G = 0;   // ring position of the current tile's K-tile 0 (mod 6)
    stage_a(G, 0);
    stage_b(G, 0);
    stage_a(G + 1, 1);
    bool first = true, prev_edge = false;
    for (;;) {
        lane = opaque_lane();
        const int nlid = lid + stride;
        const bool has_next = nlid < lid_end;
        int nm0 = m0, nn0 = n0;
        if (has_next) tile_of_lid(M, N, group, nlid, nm0, nn0);
        const int Gn = (G + nk + 1) % 6;
        const bool edge = (m0 + BM > M) || (n0 + BN > N);
        char* aux = smem + ((G + nk) % 3) * OPERAND_BYTES;
        auto load_aux = [&]() {
            if (wid == 0)
                __builtin_amdgcn_global_load_lds((gptr_t)(bias + min(n0 + lane * 4, N - 4)), (lptr_t)aux, 16, 0, 0);
            if constexpr (LN) {
                if (wid == 1)
                    __builtin_amdgcn_global_load_lds((gptr_t)(colsum + min(n0 + lane * 4, N - 4)), (lptr_t)(aux + 1024),
                                                     16, 0, 0);
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

        f32x4 acc[4][8];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

        // K-steps 0 .. nk-2: kernel 1's step (refills B(kt+1), A(kt+2) from the MFMA block; at kt = nk-2 the A
        // refill re-reads K-tile nk-1 into its own slot, identical bytes, so the block stays branch-free)
        for (int kt = 0; kt < nk - 1; ++kt) {
            if (MODE == 1 && kt == 0 && !first && !prev_edge) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
            else if (MODE == 2 && kt < 2 && !first && !prev_edge) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
            else if (MODE == 2 && kt < 2 && !first) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if (kt == nk - 2) load_aux();
            bf16x8 a[2][8], b[2][4];
            read_frags(smem + ((G + kt) % 3) * OPERAND_BYTES, smem + (3 + ((G + kt) & 1)) * OPERAND_BYTES, a, b, lane);
            stage_b(G + kt + 1, kt + 1);
            stage_a(G + min(kt + 2, nk - 1), min(kt + 2, nk - 1));
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                        acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[ks][j], a[ks][i], acc[j][i], 0, 0, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 24, 0);
            __builtin_amdgcn_sched_group_barrier(0x020, 4, 0);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            }
        }
        // K-step nk-1 (peeled): everything outstanding lands (incl. the epilogue operands); the refill is the next
        // tile's A0 into the A slot of K-tile nk-2 (free after this barrier). Without a next tile it rewrites that
        // free slot with K-tile 0 of this tile (harmless), keeping the block branch-free.
        {
            const int kt = nk - 1;
            // the builtin form: hipcc's waitcnt pass then knows no DMA is outstanding, and inserts no vmcnt(0) of its
            // own before the epilogue's LDS accesses (which would also drain the asm DMAs of the next tile)
            __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            bf16x8 a[2][8], b[2][4];
            read_frags(smem + ((G + kt) % 3) * OPERAND_BYTES, smem + (3 + ((G + kt) & 1)) * OPERAND_BYTES, a, b, lane);
            setup_a(nm0);
            stage_a_asm(Gn, 0);
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                        acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[ks][j], a[ks][i], acc[j][i], 0, 0, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 24, 0);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            }
        }

        // ---------------- epilogue ----------------
        lane = opaque_lane();
        const int tid = wid * 64 + lane;
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
        // every wave is done with K-tile nk-1's slots and the LN combine is visible
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (has_next) {
            setup_b(nn0);
            stage_b_asm(Gn, 0);        // B slot of K-tile nk-1
            stage_a_asm(Gn + 1, 1);    // A slot of K-tile nk-1
            if (MODE == 2) stage_b_asm(Gn + 1, 1);   // B slot of K-tile nk-2 (K-step 0 re-issues it: same bytes)
        }
        asm volatile("" ::: "memory");
        char* img = MODE == 2 ? aux + 16384 + wid * 2048                                 // planes consumed
                              : smem + (3 + ((G + nk) & 1)) * OPERAND_BYTES + wid * 2048;   // B slot of K-tile nk-2
        uint4 res_unused[16];
        store_wave_tile_pipe<EPI, true, false, true>(img, aux, acc, wm, wn, m0, n0, lane, res_unused, C, ldc, M, N,
                                                     nullptr, 0);
        if (!has_next) break;
        first = false;
        prev_edge = edge;
        lid = nlid;
        m0 = nm0;
        n0 = nn0;
        G = Gn;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may outlive the workgroup
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

    const char* Ablk = reinterpret_cast<const char*>(A) + (size_t)m0 * lda * 2;
    const char* Bblk = reinterpret_cast<const char*>(W) + (size_t)n0 * K * 2;
    // per-lane DMA source offsets: [type][piece]; piece p of a half-tile = local rows (wid + 8p) * 8 + lane / 8
    uint32_t off[4][2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int rho = (wid + 8 * p) * 8 + (lane >> 3);             // local row 0..127
        const int lch = (lane & 7) ^ ((rho >> 1) & 7);               // logical chunk at this physical slot
        const int ra0 = (rho >> 6) * 128 + (rho & 63);               // A0: g*128 + r
        const int rb0 = (rho >> 5) * 64 + (rho & 31);                // B0: wn*64 + r
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

// ---------------------------------------------------------------------------------------------------------------
// Four-wave variant (hipBLASLt's gfx950 shape: 256 threads, each wave a 128 x 128 sub-tile with its 256 fp32
// accumulators in AGPRs, one wave per SIMD): half the LDS fragment bytes per MFMA of the 8-wave kernel.
//  * Same 256x256x64 tile, swizzled LDS image, deep ring (A slots 0-2, B slots 3-4) and XCD-aware tile order as
//    k_gemm_bf16. A K-tile's two 32-deep slices are the two MFMA phases of one loop iteration:
//      phase A: 64 MFMAs on slice 0 (fragments F0_t in registers), the 16 fragment reads of slice 1 (F1_t)
//               interleaved one per 4 MFMAs;
//      lgkmcnt(0), vmcnt(8), ONE barrier Y_t (K-tile t+1 landed for every wave; every wave's reads of K-tile t
//               are retired);
//      phase B: 64 MFMAs on slice 1 (F1_t), the 16 reads of K-tile t+1's slice 0 (F0_{t+1}) and the 16 DMA
//               pieces B(t+2), A(t+3) interleaved. Both refills go to the slots of K-tile t, whose last reads
//               (F1_t) were retired before Y_t. Lookahead: B one K-tile, A two.
//  * vmcnt(8) at Y_t leaves A(t+2) (issued last, in phase B of t-1) in flight and retires B(t+1), A(t+1).
//  * Past the end the refills re-read K-tile nk-1 into its own slots (identical bytes) and the phase-B reads of
//    K-tile nk read unused bytes, so the loop body is branch-free. The epilogue operands land in A slot nk % 3
//    (K-tile nk-3's, free after Y_{nk-3}), issued after Y_{nk-2}; the epilogue images use the B slots.
//  * hipcc does not keep 256 builtin-MFMA accumulators resident in AGPRs (it copies every C operand through
//    a[0:3]), so the MFMAs, fragment reads and their waits are inline asm (cdna_hip_programming.md §5.7): "+a"
//    accumulators, lds16 reads retired by explicit lgkmcnt(0) statements that name their registers, the first
//    slice with C = 0 (no AGPR zero-fill), and the MFMA -> VALU hazard padded before the epilogue reads.
//  * Epilogue: the 8-wave epilogue functions, once per 64-column half (wn' = 2 wn + h).
__device__ __forceinline__ void mfma_acc(f32x4& c, const i32x4& w, const i32x4& x) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(w), "v"(x));
}
__device__ __forceinline__ void mfma_zero(f32x4& c, const i32x4& w, const i32x4& x) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(w), "v"(x));
}
// lgkmcnt(0) that the compiler sees as writing the named fragment registers: no copy of them can be scheduled
// between their lds16 reads and this wait (§5.7 item 1, form ii)
#define VPF_W4_WAIT16(A, B)                                                                                          \
    asm volatile("s_waitcnt lgkmcnt(0)"                                                                          \
                 : "+v"(A[0]), "+v"(A[1]), "+v"(A[2]), "+v"(A[3]), "+v"(A[4]), "+v"(A[5]), "+v"(A[6]), "+v"(A[7]), \
                   "+v"(B[0][0]), "+v"(B[0][1]), "+v"(B[0][2]), "+v"(B[0][3]), "+v"(B[1][0]), "+v"(B[1][1]),        \
                   "+v"(B[1][2]), "+v"(B[1][3])::"memory")

// BAL: A(t+2) is issued in phase A of K-tile t (8 pieces per phase) instead of A(t+3) in phase B; the prologue then
// stages A0 B0 A1 B1 and the vmcnt count at Y_t is the same (A(t+2), issued after B(t+1)... see phase_a).
// NOEPI (lab kernel 28): the K loop alone, no epilogue (timing probe; C not written).
template <int EPI, bool OUT8 = false, bool BAL = true, bool NOEPI = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void k_gemm_w4(const bf16_t* __restrict__ A, int lda, const bf16_t* __restrict__ W, const float* __restrict__ bias,
               const bf16_t* residual, const float* __restrict__ pos, int g2, const float2* __restrict__ stats,
               const float* __restrict__ colsum, bf16_t* C, int ldc, int M, int N, int K, int group, int stats_parts,
               float ln_eps, float* stats_out, int stats_rows, Out8 o8) {
    __shared__ __attribute__((aligned(16))) char smem[5 * OPERAND_BYTES];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid >> 1, wn = wid & 1;
    int m0, n0;
    tile_of(M, N, group, m0, n0);
    const char* Ablk = reinterpret_cast<const char*>(A) + (size_t)m0 * lda * 2;
    const char* Bblk = reinterpret_cast<const char*>(W) + (size_t)n0 * K * 2;
    uint32_t offA[8], offB[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int row = 8 * (i * 4 + wid) + (lane >> 3);
        const int lch = (lane & 7) ^ ((row >> 1) & 7);
        offA[i] = (uint32_t)min(row, M - 1 - m0) * (uint32_t)(lda * 2) + (uint32_t)(lch * 16);
        offB[i] = (uint32_t)min(row, N - 1 - n0) * (uint32_t)(K * 2) + (uint32_t)(lch * 16);
    }
    const int nk = K / BK;
    auto dma_a = [&](int kt, int i) {
        __builtin_amdgcn_global_load_lds((gptr_t)(Ablk + offA[i] + (uint32_t)kt * (BK * 2)),
                                         (lptr_t)(smem + (kt % 3) * OPERAND_BYTES + (i * 4 + wid) * 1024), 16, 0, 0);
    };
    auto dma_b = [&](int kt, int i) {
        __builtin_amdgcn_global_load_lds((gptr_t)(Bblk + offB[i] + (uint32_t)kt * (BK * 2)),
                                         (lptr_t)(smem + (3 + (kt & 1)) * OPERAND_BYTES + (i * 4 + wid) * 1024), 16, 0,
                                         0);
    };
    constexpr bool LN = (EPI == VPF_EPI_LN || EPI == VPF_EPI_LN_GELU);
    char* aux = smem + (nk % 3) * OPERAND_BYTES;
    auto load_aux = [&]() {   // k_gemm_bf16's aux layout, pieces dealt over 4 waves (<= 8 per wave)
        if (wid == 0)
            __builtin_amdgcn_global_load_lds((gptr_t)(bias + min(n0 + lane * 4, N - 4)), (lptr_t)aux, 16, 0, 0);
        if constexpr (LN) {
            if (wid == 1)
                __builtin_amdgcn_global_load_lds((gptr_t)(colsum + min(n0 + lane * 4, N - 4)), (lptr_t)(aux + 1024), 16,
                                                 0, 0);
            const float* sd = reinterpret_cast<const float*>(stats);
            const int planes = stats_parts > 0 ? stats_parts : 1;
            if ((M & 1) == 0 && ((uintptr_t)sd & 15) == 0) {
                for (int pc = wid; pc < 2 * planes; pc += 4) {
                    const int p = pc >> 1, hf = pc & 1;
                    __builtin_amdgcn_global_load_lds(
                        (gptr_t)(sd + (int64_t)p * 2 * M + min(2 * m0 + hf * 256 + lane * 4, 2 * M - 4)),
                        (lptr_t)(aux + 2048 + p * 2048 + hf * 1024), 16, 0, 0);
                }
            } else {
                for (int p = 0; p < planes; ++p)
#pragma unroll
                    for (int q = 0; q < 2; ++q)
                        __builtin_amdgcn_global_load_lds(
                            (gptr_t)(sd + (int64_t)p * 2 * M + min(2 * m0 + (wid * 2 + q) * 64 + lane, 2 * M - 1)),
                            (lptr_t)(aux + 2048 + p * 2048 + (wid * 2 + q) * 256), 4, 0, 0);
            }
        }
    };

    // fragment reads: A rows wm*128 + i*16 + fr (i < 8), B (W) rows wn*128 + (h*4 + j)*16 + fr; slice ks = logical
    // chunk ks*4 + fq of the 128-B row
    const int fr = lane & 15, fq = lane >> 4;
    const int sw = (fr >> 1) & 7;
    const int arow = (wm * 128 + fr) * 128, brow = (wn * 128 + fr) * 128;
    auto slice_base = [&](int kt, int ks, const char*& la, const char*& lb) {
        la = smem + (kt % 3) * OPERAND_BYTES + arow + (((ks * 4 + fq) ^ sw) << 4);
        lb = smem + (3 + (kt & 1)) * OPERAND_BYTES + brow + (((ks * 4 + fq) ^ sw) << 4);
    };
    // fragment q (0..15) of a slice: q < 8 -> A fragment q, else B fragment (h, j) = ((q-8) >> 2, (q-8) & 3)
    auto read_frag = [&](i32x4 (&a)[8], i32x4 (&b)[2][4], const char* la, const char* lb, int q) {
        if (q < 8) a[q] = lds16(la + q * 2048);
        else b[(q - 8) >> 2][(q - 8) & 3] = lds16(lb + (q - 8) * 2048);
    };

    f32x4 acc[2][4][8];
    i32x4 a0[8], b0[2][4], a1[8], b1[2][4];

    // prologue: A0 B0 A1 B1 A2 (8 pieces each); K-tile 0 landed = all but the 24 youngest pieces
#pragma unroll
    for (int i = 0; i < 8; ++i) dma_a(0, i);
#pragma unroll
    for (int i = 0; i < 8; ++i) dma_b(0, i);
#pragma unroll
    for (int i = 0; i < 8; ++i) dma_a(min(1, nk - 1), i);
#pragma unroll
    for (int i = 0; i < 8; ++i) dma_b(min(1, nk - 1), i);
    if constexpr (!BAL) {
#pragma unroll
        for (int i = 0; i < 8; ++i) dma_a(min(2, nk - 1), i);
    }
    if (nk == 1) load_aux();   // slot 1: no K-tile uses it
    if constexpr (BAL) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    {
        const char *la, *lb;
        slice_base(0, 0, la, lb);
#pragma unroll
        for (int q = 0; q < 16; ++q) read_frag(a0, b0, la, lb, q);
    }

    // phase A: MFMAs of slice 0 (a0/b0) with slice 1's reads (a1/b1) of K-tile kt interleaved, then the barrier
    auto phase_a = [&](int kt, auto first) {
        VPF_W4_WAIT16(a0, b0);
        const char *la, *lb;
        slice_base(kt, 1, la, lb);
        const int ka = min(kt + 2, nk - 1);   // BAL: A(kt+2) -> the slot of K-tile kt-1 (free after Y_{kt-1})
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    if constexpr (decltype(first)::value) mfma_zero(acc[h][j][i], b0[h][j], a0[i]);
                    else mfma_acc(acc[h][j][i], b0[h][j], a0[i]);
                    if ((i & 3) == 3) {
                        const int q = (h * 4 + j) * 2 + (i >> 2);
                        read_frag(a1, b1, la, lb, q);
                        if (BAL && (q & 1)) dma_a(ka, q >> 1);
                    }
                }
            }
        VPF_W4_WAIT16(a1, b1);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    };
    // phase B: MFMAs of slice 1 (a1/b1) with K-tile kt+1's slice-0 reads and the B(kt+2), A(kt+3) refills
    auto phase_b = [&](int kt) {
        if (kt == nk - 2) load_aux();
        const char *la, *lb;
        slice_base(kt + 1, 0, la, lb);
        const int kb = min(kt + 2, nk - 1), ka = min(kt + 3, nk - 1);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    mfma_acc(acc[h][j][i], b1[h][j], a1[i]);
                    if ((i & 3) == 3) {
                        const int q = (h * 4 + j) * 2 + (i >> 2);
                        read_frag(a0, b0, la, lb, q);
                        if (BAL) { if (q & 1) dma_b(kb, q >> 1); }
                        else if (q < 8) dma_b(kb, q);
                        else dma_a(ka, q - 8);
                    }
                }
            }
    };
    phase_a(0, std::true_type{});
    phase_b(0);
    for (int kt = 1; kt < nk; ++kt) {
        phase_a(kt, std::false_type{});
        phase_b(kt);
    }
    VPF_W4_WAIT16(a0, b0);   // the unused reads of "K-tile nk"
    // MFMA -> VALU / v_accvgpr_read hazard (§5.7 item 2: up to 12 wait states); the statements name every
    // accumulator, so no reader of one is scheduled above them
    asm volatile("s_nop 7\n\ts_nop 7" : "+a"(acc[0][0][0]), "+a"(acc[0][0][1]), "+a"(acc[0][0][2]), "+a"(acc[0][0][3]),
                 "+a"(acc[0][0][4]), "+a"(acc[0][0][5]), "+a"(acc[0][0][6]), "+a"(acc[0][0][7]));
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            asm volatile("" : "+a"(acc[h][j][0]), "+a"(acc[h][j][1]), "+a"(acc[h][j][2]), "+a"(acc[h][j][3]),
                         "+a"(acc[h][j][4]), "+a"(acc[h][j][5]), "+a"(acc[h][j][6]), "+a"(acc[h][j][7]));

    if constexpr (NOEPI) {
        __builtin_amdgcn_s_waitcnt(0x0F70);
        return;
    }
    // ---------------- epilogue ----------------
    if constexpr (LN) {
        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the epilogue operands landed ...
        __builtin_amdgcn_s_barrier();         // ... for every wave
        if (stats_parts > 0) {               // tid < 256 = BM: one row per thread
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
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    constexpr bool PIPE = EPI != VPF_EPI_PATCH && !OUT8;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    char* img = smem + 3 * OPERAND_BYTES + wid * 16384;   // B slots: never the aux slot
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        uint4 res[16];
        if constexpr (EPI == VPF_EPI_BIAS_RESIDUAL) load_residual<PIPE>(res, residual, wm, 2 * wn + h, m0, n0, lane, ldc, M, N);
        if constexpr (PIPE) {
            store_wave_tile_pipe<EPI>(img, aux, acc[h], wm, 2 * wn + h, m0, n0, lane, res, C, ldc, M, N,
                                      EPI == VPF_EPI_BIAS_RESIDUAL ? stats_out : nullptr, stats_rows);
        } else {
            float* prod_stats = (EPI == VPF_EPI_BIAS_RESIDUAL || EPI == VPF_EPI_PATCH) ? stats_out : nullptr;
            store_wave_tile<EPI, OUT8>(img, aux, acc[h], wm, 2 * wn + h, m0, n0, lane, res, pos, g2, C, ldc, M, N,
                                       prod_stats, stats_rows, o8);
        }
        __builtin_amdgcn_wave_barrier();   // the wave's image is reused by the second half (LDS ops stay in order)
    }
}

}  // namespace

#define VPF_IS_LN(E) ((E) == VPF_EPI_LN || (E) == VPF_EPI_LN_GELU)
#define VPF_IS_PROD(E) ((E) == VPF_EPI_BIAS_RESIDUAL || (E) == VPF_EPI_PATCH)
#define VPF_GEMM_ARGS                                                                                        \
    A, (int)lda, W, bias, residual, pos, patch_rows, reinterpret_cast<const float2*>(row_stats), colsum, C,     \
        (int)ldc, m, n, k, group, stats_parts, ln_eps, stats_out, stats_rows, o8
// fp8 copies are produced by the residual-stream producers only (proj, patch embed): the only bf16 GEMMs
// whose output an MX8 GEMM reads
#define VPF_GEMM_PT_OK(E) ((E) == VPF_EPI_LN || (E) == VPF_EPI_LN_GELU || (E) == VPF_EPI_BIAS || (E) == VPF_EPI_BIAS_GELU)
// Kernels 8 / 9 (LAB 1 / 2: the C stores predicated off / no epilogue at all) never write their output: timing-only
// variants, compiled into lab builds alone (-DVPF_GEMM_LAB, tools/gemm_lab). A product build rejects them in
// vpf_gemm_tune and ignores them in VPF_GEMM_KERNEL.
#ifdef VPF_GEMM_LAB
constexpr bool kGemmLab = true;
static int gemm_pf_dist() {   // kernel 27's prefetch distance in K-tiles (VPF_GEMM_PFD, default 4)
    const char* e = getenv("VPF_GEMM_PFD");
    const int d = e ? atoi(e) : 4;
    return d < 1 ? 1 : d > 15 ? 15 : d;
}
#define VPF_GEMM_LAB_LAUNCH(E)                                                                               \
    else if ((kern == 8 || kern == 9) && !(VPF_IS_LN(E) && stats_parts > AUX_PARTS) && o8.q == nullptr) {    \
        if (kern == 8)                                                                                       \
            hipLaunchKernelGGL((k_gemm_bf16<E, true, false, false, true, true, true, 1>), grid, block, 0, s,   \
                               A, (int)lda, W, bias, residual, pos, patch_rows,                               \
                               reinterpret_cast<const float2*>(row_stats), colsum, C, (int)ldc, m, n, k,        \
                               group | 0x10000, stats_parts, ln_eps, stats_out, stats_rows, o8);              \
        else                                                                                                 \
            hipLaunchKernelGGL((k_gemm_bf16<E, true, false, false, true, true, true, 2>), grid, block, 0, s,   \
                               A, (int)lda, W, bias, residual, pos, patch_rows,                               \
                               reinterpret_cast<const float2*>(row_stats), colsum, C, (int)ldc, m, n, k,        \
                               group | 0x10000, stats_parts, ln_eps, stats_out, stats_rows, o8);              \
    }                                                                                                        \
    else if (kern == 28 && !(VPF_IS_LN(E) && stats_parts > AUX_PARTS) && o8.q == nullptr) {                 \
        hipLaunchKernelGGL((k_gemm_w4<E, false, true, true>), grid, dim3(256), 0, s, VPF_GEMM_ARGS);           \
    }                                                                                                        \
    else if (kern == 29 && !(VPF_IS_LN(E) && stats_parts > AUX_PARTS) && o8.q == nullptr) {                 \
        hipLaunchKernelGGL((k_gemm_bf16<E, true, false, false, true, true, true, 13>), grid, block, 0, s,      \
                           VPF_GEMM_ARGS);                                                                   \
    }                                                                                                        \
    else if (kern >= 30 && kern <= 32 && !(VPF_IS_LN(E) && stats_parts > AUX_PARTS) && o8.q == nullptr) {    \
        if (kern == 30)                                                                                      \
            hipLaunchKernelGGL((k_gemm_bf16<E, true, false, false, true, true, true, 14>), grid, block, 0, s,  \
                               VPF_GEMM_ARGS);                                                               \
        else if (kern == 31)                                                                                 \
            hipLaunchKernelGGL((k_gemm_bf16<E, true, false, false, true, true, true, 15>), grid, block, 0, s,  \
                               VPF_GEMM_ARGS);                                                               \
        else                                                                                                 \
            hipLaunchKernelGGL((k_gemm_bf16<E, true, false, false, true, true, true, 16>), grid, block, 0, s,  \
                               VPF_GEMM_ARGS);                                                               \
    }                                                                                                        \
    else if (kern == 27 && !(VPF_IS_LN(E) && stats_parts > AUX_PARTS) && o8.q == nullptr) {                 \
        hipLaunchKernelGGL((k_gemm_bf16<E, true, false, false, true, true, true, 12>), grid, block, 0, s,      \
                           A, (int)lda, W, bias, residual, pos, patch_rows,                                   \
                           reinterpret_cast<const float2*>(row_stats), colsum, C, (int)ldc, m, n, k,            \
                           group | (gemm_pf_dist() << 17), stats_parts, ln_eps, stats_out, stats_rows, o8);   \
    }                                                                                                        \
    else if (kern >= 24 && kern <= 26 && !(VPF_IS_LN(E) && stats_parts > AUX_PARTS) && o8.q == nullptr) {    \
        if (kern == 24)                                                                                      \
            hipLaunchKernelGGL((k_gemm_bf16<E, true, false, false, true, true, true, 9>), grid, block, 0, s,   \
                               VPF_GEMM_ARGS);                                                               \
        else if (kern == 25)                                                                                 \
            hipLaunchKernelGGL((k_gemm_bf16<E, true, false, false, true, true, true, 10>), grid, block, 0, s,  \
                               VPF_GEMM_ARGS);                                                               \
        else                                                                                                 \
            hipLaunchKernelGGL((k_gemm_bf16<E, true, false, false, true, true, true, 11>), grid, block, 0, s,  \
                               VPF_GEMM_ARGS);                                                               \
    }                                                                                                        \
    else if (kern >= 20 && kern <= 23 && !(VPF_IS_LN(E) && stats_parts > AUX_PARTS) && o8.q == nullptr) {    \
        if (kern == 20)                                                                                      \
            hipLaunchKernelGGL((k_gemm_bf16<E, true, false, false, true, true, true, 5>), grid, block, 0, s,   \
                               VPF_GEMM_ARGS);                                                               \
        else if (kern == 21)                                                                                 \
            hipLaunchKernelGGL((k_gemm_bf16<E, true, false, false, true, true, true, 6>), grid, block, 0, s,   \
                               VPF_GEMM_ARGS);                                                               \
        else if (kern == 22)                                                                                 \
            hipLaunchKernelGGL((k_gemm_bf16<E, true, false, false, true, true, true, 7>), grid, block, 0, s,   \
                               VPF_GEMM_ARGS);                                                               \
        else                                                                                                 \
            hipLaunchKernelGGL((k_gemm_bf16<E, true, false, false, true, true, true, 8>), grid, block, 0, s,   \
                               VPF_GEMM_ARGS);                                                               \
    }
#else
constexpr bool kGemmLab = false;
#define VPF_GEMM_LAB_LAUNCH(E)
#endif
static bool gemm_kernel_ok(int k) {
    return (k >= 1 && k <= 17 && (kGemmLab || (k != 8 && k != 9))) || (kGemmLab && k >= 20 && k <= 32);
}
#define VPF_GEMM_LAUNCH(E)                                                                                   \
    do {                                                                                                     \
        if constexpr (VPF_GEMM_PT_OK(E)) {                                                                   \
            if (kern >= 13 && kern <= 15 && stats_parts <= AUX_PARTS && o8.q == nullptr && k >= 2 * BK) {     \
                const unsigned pg = (unsigned)std::min<int64_t>((tiles + 7) & ~7, (int64_t)(gemm_cus() & ~7)); \
                if (kern == 13)                                                                              \
                    hipLaunchKernelGGL((k_gemm_pt<VPF_GEMM_PT_OK(E) ? E : VPF_EPI_BIAS>), dim3(pg), block, 0, s, A, \
                                       (int)lda, W, bias, reinterpret_cast<const float2*>(row_stats), colsum, C, \
                                       (int)ldc, m, n, k, group, stats_parts, ln_eps);                       \
                else if (kern == 15)                                                                         \
                    hipLaunchKernelGGL((k_gemm_pt<VPF_GEMM_PT_OK(E) ? E : VPF_EPI_BIAS, 2>), dim3(pg), block, 0, \
                                       s, A, (int)lda, W, bias, reinterpret_cast<const float2*>(row_stats), colsum, \
                                       C, (int)ldc, m, n, k, group, stats_parts, ln_eps);                    \
                else                                                                                         \
                    hipLaunchKernelGGL((k_gemm_pt<VPF_GEMM_PT_OK(E) ? E : VPF_EPI_BIAS, 0>), dim3(pg), block, 0, \
                                       s, A, (int)lda, W, bias, reinterpret_cast<const float2*>(row_stats), colsum, \
                                       C, (int)ldc, m, n, k, group, stats_parts, ln_eps);                    \
                break;                                                                                       \
            }                                                                                                \
        }                                                                                                    \
        if (kern == 16 && !(VPF_IS_LN(E) && stats_parts > AUX_PARTS) && o8.q == nullptr) {                  \
            hipLaunchKernelGGL((k_gemm_bf16<E, true, false, false, true, true, true, 4>), grid, block, 0, s,   \
                               VPF_GEMM_ARGS);                                                               \
        } else if (kern >= 10 && kern <= 12 && !(VPF_IS_LN(E) && stats_parts > AUX_PARTS) && o8.q == nullptr) { \
            hipLaunchKernelGGL((k_gemm_bf16<E, true, false, false, true, true, true, 3>), grid, block, 0, s,   \
                               A, (int)lda, W, bias, residual, pos, patch_rows,                               \
                               reinterpret_cast<const float2*>(row_stats), colsum, C, (int)ldc, m, n, k,        \
                               group | ((kern == 10 ? 2 : kern == 11 ? 1 : 3) << 17), stats_parts, ln_eps,     \
                               stats_out, stats_rows, o8);                                                    \
        }                                                                                                    \
        VPF_GEMM_LAB_LAUNCH(E)                                                                               \
        else if (kern == 17) {                                                                               \
            if (VPF_IS_LN(E) && stats_parts > AUX_PARTS)                                                     \
                hipLaunchKernelGGL((k_gemm_bf16<E, true, VPF_IS_LN(E), false, true, true, true, 0, false, true>), \
                                   grid, block, 0, s, VPF_GEMM_ARGS);                                        \
            else if (VPF_IS_PROD(E) && o8.q != nullptr)                                                      \
                hipLaunchKernelGGL((k_gemm_bf16<E, true, false, VPF_IS_PROD(E), true, true, true, 0, false, true>), \
                                   grid, block, 0, s, VPF_GEMM_ARGS);                                        \
            else                                                                                             \
                hipLaunchKernelGGL((k_gemm_bf16<E, true, false, false, true, true, true, 0, false, true>), grid, \
                                   block, 0, s, VPF_GEMM_ARGS);                                              \
        }                                                                                                    \
        else if (kern == 2)                                                                                  \
            hipLaunchKernelGGL((k_gemm_bf16<E, false>), grid, block, 0, s, VPF_GEMM_ARGS);                    \
        else if (kern == 3 && !(VPF_IS_LN(E) && stats_parts > AUX_PARTS) && !(VPF_IS_PROD(E) && o8.q))       \
            hipLaunchKernelGGL((k_gemm_bf16<E, true, false, false, false>), grid, block, 0, s, VPF_GEMM_ARGS); \
        else if (kern == 4 && !(VPF_IS_LN(E) && stats_parts > AUX_PARTS) && !(VPF_IS_PROD(E) && o8.q))       \
            hipLaunchKernelGGL((k_gemm_bf16<E, true, false, false, true, false>), grid, block, 0, s, VPF_GEMM_ARGS); \
        else if (kern == 7 && !(VPF_IS_LN(E) && stats_parts > AUX_PARTS) && o8.q == nullptr)                \
            hipLaunchKernelGGL((k_gemm_w4<E, false>), grid, dim3(256), 0, s, VPF_GEMM_ARGS);                   \
        else if (kern == 7 && !(VPF_IS_LN(E) && stats_parts > AUX_PARTS) && VPF_IS_PROD(E))                 \
            hipLaunchKernelGGL((k_gemm_w4<E, VPF_IS_PROD(E)>), grid, dim3(256), 0, s, VPF_GEMM_ARGS);          \
        else if (kern == 6 && !(VPF_IS_LN(E) && stats_parts > AUX_PARTS) && !(VPF_IS_PROD(E) && o8.q))       \
            hipLaunchKernelGGL((k_gemm_bf16<E, true, false, false, true, true, false>), grid, block, 0, s, VPF_GEMM_ARGS); \
        else if (kern == 5 && !(VPF_IS_LN(E) && stats_parts > AUX_PARTS) && o8.q == nullptr)                \
            hipLaunchKernelGGL((k_gemm_pp<E, false>), grid, block, 0, s, VPF_GEMM_ARGS);                     \
        else if (kern == 5 && VPF_IS_PROD(E) && o8.q != nullptr)                                             \
            hipLaunchKernelGGL((k_gemm_pp<E, VPF_IS_PROD(E)>), grid, block, 0, s, VPF_GEMM_ARGS);            \
        else if (VPF_IS_LN(E) && stats_parts > AUX_PARTS)                                                    \
            hipLaunchKernelGGL((k_gemm_bf16<E, true, VPF_IS_LN(E)>), grid, block, 0, s, VPF_GEMM_ARGS);       \
        else if (VPF_IS_PROD(E) && o8.q != nullptr)                                                          \
            hipLaunchKernelGGL((k_gemm_bf16<E, true, false, VPF_IS_PROD(E)>), grid, block, 0, s, VPF_GEMM_ARGS); \
        else                                                                                                 \
            hipLaunchKernelGGL((k_gemm_bf16<E, true>), grid, block, 0, s, VPF_GEMM_ARGS);                     \
    } while (0)

static int gemm_cus() {   // compute units of the current device (the persistent kernel's grid)
    static int cached = 0;
    if (!cached) {
        int dev = 0, n = 0;
        cached = (hipGetDevice(&dev) == hipSuccess &&
                  hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n >= 8) ? n : 256;
    }
    return cached;
}

static int g_group = -1;
static bool g_group_set = false;   // VPF_GEMM_GROUP or vpf_gemm_tune set one group for every shape
static int tile_group() {   // VPF_GEMM_GROUP overrides the A-panel group size of the tile order (0 = tm-major)
    if (g_group < 0) {
        const char* e = getenv("VPF_GEMM_GROUP");
        g_group = e ? atoi(e) : 4;
        g_group_set = e != nullptr;
        if (g_group < 0) g_group = 0;
    }
    return g_group;
}
// Default group per shape (profiles/r2_gemm_lab/group_sweep_r2.txt, one process): the N <= 1024 GEMMs (proj / FC2:
// 3 column tiles, so a group of 4 A panels keeps 12 tiles of one K panel set in flight) are 1-1.5 % faster with 2
// panels per group (FC2 3.196 vs 3.226 ms, proj 1.070 vs 1.082), QKV / FC1 with 4. The order never changes a bit.
// FC1 (EPI_LN_GELU; 12 column tiles at ViT-B) takes 8 A panels per group: 16 was -0.9 % on FC1 and -0.7 % on the frame
// against 4 in a same-box A/B (profiles/r2_gemm_lab/fc1_group16_pmc.txt), and 8 is another 0.3-0.5 % ahead of 16 in
// two one-process sweeps (group_sweep_r2s5.txt, fc1_pp_group_ab.txt).
static int tile_group_for(int64_t N, int epilogue) {
    const int g = tile_group();
    if (g_group_set) return g;
    if (N <= 1024) return 2;
    return epilogue == VPF_EPI_LN_GELU ? 8 : g;
}

// GEMM kernel selection: 1 = k_gemm_bf16 with the deep A ring, refills issued from the MFMA block (product);
// 2 = the 2-stage ring, 3 = the deep ring with both refills issued right after the barrier, 4 = kernel 1 with the
// two-pass epilogue, 5 = the ping-pong loop k_gemm_pp, 6 = kernel 1 with the original epilogue row order, 7 = the
// four-wave k_gemm_w4, 8 / 9 = kernel 1 without its C stores / without its epilogue (A/B timing; outputs not written;
// -DVPF_GEMM_LAB builds only), 10 / 11 / 12 = kernel 1
// with a staggered start in 4 / 2 / 8 phases, 13 = the persistent k_gemm_pt (LN / LN_GELU / BIAS / BIAS_GELU; else 1).
// VPF_GEMM_KERNEL sets the initial value, vpf_gemm_tune() the current one.
static int g_kernel = -1;
static bool g_kernel_set = false;   // VPF_GEMM_KERNEL or vpf_gemm_tune chose one kernel for every shape
static int gemm_kernel() {
    if (g_kernel < 0) {
        const char* e = getenv("VPF_GEMM_KERNEL");
        g_kernel = e ? atoi(e) : 1;
        g_kernel_set = e != nullptr;
        if (!gemm_kernel_ok(g_kernel)) { g_kernel = 1; g_kernel_set = false; }
    }
    return g_kernel;
}
// Default kernel per epilogue: the LN-folded bias-only GEMM (QKV) runs the ping-pong loop k_gemm_pp (kernel 5), 2.5 %
// faster there in one process (2.603 vs 2.670 ms, profiles/r2_gemm_lab/kernel_ab_r2s5.txt) and bit-identical to
// kernel 1 (test_gemm_kernel_variants_bit_identical); every other epilogue is fastest on kernel 1.
static int gemm_kernel_for(int epilogue) {
    const int k = gemm_kernel();
    return g_kernel_set ? k : (epilogue == VPF_EPI_LN ? 5 : k);
}
int vpf_gemm_tile_group() { return tile_group(); }   // shared with gemm_mx8.hip
// MX8 GEMMs' default group (profiles/r2_gemm_lab/mx8_group_sweep.txt, fp8 frames): the LN-folded bias-only QKV is ~5 %
// faster with 8 A panels per group (1.93-1.95 vs 2.05 ms); proj / FC1 / FC2 keep 4.
int vpf_gemm_tile_group_mx8(int epilogue) {
    const int g = tile_group();
    return g_group_set ? g : (epilogue == VPF_EPI_LN ? 8 : g);
}
VPF_API int vpf_gemm_tune(int kernel, int group) {
    if (kernel != 0 && !gemm_kernel_ok(kernel)) return VPF_ERR_ARG;
    gemm_kernel();
    tile_group();
    if (kernel == 0) {   // back to the per-shape defaults (kernel and group)
        g_kernel = 1; g_kernel_set = false;
        g_group = 4; g_group_set = false;
        return 0;
    }
    g_kernel = kernel;
    g_kernel_set = true;
    if (group >= 0) { g_group = group; g_group_set = true; }
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
    if (stats_parts < 0 || stats_parts > (gemm_kernel() == 2 ? AUX_PARTS : MAX_PARTS) || !(ln_eps >= 0.f))
        return VPF_ERR_ARG;
    if (stats_out && (((uintptr_t)stats_out & 7) || (epilogue != VPF_EPI_BIAS_RESIDUAL && epilogue != VPF_EPI_PATCH)))
        return VPF_ERR_ARG;
    // producer plane stride: rows of C (EPI_PATCH interleaves one CLS row per patch_rows rows)
    const int64_t srows = epilogue == VPF_EPI_PATCH ? (M / patch_rows) * (patch_rows + 1) : M;
    if (srows > INT32_MAX) return VPF_ERR_ARG;
    const int stats_rows = (int)srows;
    // fp8 copy of C: residual-stream producers only, deep-ring kernel
    if (C8 && ((epilogue != VPF_EPI_BIAS_RESIDUAL && epilogue != VPF_EPI_PATCH) || gemm_kernel() == 2))
        return VPF_ERR_ARG;
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
    hipLaunchKernelGGL((k_gemm_bf16<VPF_EPI_BIAS, true, false, false, true, true, true, 0, true>),
                       dim3((unsigned)tiles, (unsigned)splits), dim3(NTHREADS), 0, s, reinterpret_cast<const bf16_t*>(A),
                       (int)lda, reinterpret_cast<const bf16_t*>(W), nullptr, nullptr, nullptr, 1, nullptr, nullptr,
                       reinterpret_cast<bf16_t*>(partial_ws), n, m, n, k, tile_group(), 0, 0.f, nullptr, m, o8);
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
