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
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "vpf_common.h"
#include "mx8.h"
#include "../../include/vpf.h"

using namespace vpf;

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

typedef const __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

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

// max / sum of a value with its partner lane l ^ 32 by one v_permlane32_swap (VALU, no LDS round trip; the
// __shfl_xor form costs a ds_bpermute, its address VALU and an lgkmcnt wait on the step's critical path).
// Every lane of the wave must be active.
__device__ __forceinline__ float xor32_max(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    float y;   // one v_max_f32: fmaxf on bit-cast values adds two NaN-canonicalising v_max (scores are never NaN)
    asm("v_max_f32 %0, %1, %2" : "=v"(y) : "v"(__uint_as_float(r[0])), "v"(__uint_as_float(r[1])));
    return y;
}
__device__ __forceinline__ float xor32_sum(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// One key step of T 32-key tiles (T = 1 or 2) for a 32-query strip: S^T = K Q^T on MFMA, online softmax
// update of (m, l, O), O^T += V^T P^T with V^T fragments from transposed LDS reads. MASK: this step contains
// padded keys (only the last step). The O / l rescale is skipped when no query's running max moved in this
// step (wave-uniform test), which is the common case after the first key tiles.
// ds_read_b64_tr_b16 as inline asm: hipcc treats the builtin as a possible reader of in-flight LDS-DMA
// bytes and drains vmcnt(0) before it, which would serialise the key-pipelined kernel on its last chunk.
// The caller waits lgkmcnt itself (tr_wait) before the MFMA that consumes the result.
// A constant byte offset goes in the instruction's offset field. V rows r + 8 and r + 16 keep bit 1
// of r, so v_off(r + 8j, c) = v_off(r, c) + 1024 j: the four row blocks of a key step share one address VGPR
// per 32-dim column tile instead of one v_add each.
template <int OFF>
__device__ __forceinline__ bf16x4 ds_read_tr_asm_o(uint32_t addr) {
    bf16x4 r;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
    return r;
}

#ifndef VPF_ATTN_VEARLY   // -DVPF_ATTN_VEARLY=1: PRE also issues the first V^T tile's reads early (spills; A/B only)
#define VPF_ATTN_VEARLY 0
#endif
// PRE (ASM_TR only): the four K fragment reads are issued together ahead of the QK^T MFMAs, and the eight V^T reads
// right behind those MFMAs, so their LDS latency runs under the softmax VALU instead of after it.
template <int T, bool MASK, bool ASM_TR = false, bool PRE = false>
__device__ __forceinline__ void attn_step(const char* Ks, const char* Vs, int kb, int N, int lane, const bf16x8 qf[4],
                                          float scale_log2, float& m, float& l, f32x16& o0, f32x16& o1) {
    static_assert(!PRE || (ASM_TR && T == 1), "PRE: the one-tile asm transposed-read step");
    const int l32 = lane & 31, hh = lane >> 5;
    f32x16 s[T];
    bf16x4 vr[2][2][2];
    if constexpr (PRE) {
        s[0] = f32x16{};
        const int kr = kb + l32;
        bf16x8 kf[4];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) kf[ks] = *reinterpret_cast<const bf16x8*>(Ks + k_off(kr, ks * 2 + hh));
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) s[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[ks], qf[ks], s[0], 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_barrier(0);
        const int grp = lane >> 4, gi = lane & 15;
        const int rbase = kb + 4 * (grp >> 1) + (gi >> 2);
        if constexpr (VPF_ATTN_VEARLY) {   // the first 32-dim column tile's V^T reads (8 VGPRs; both tiles' 16 spill)
            const int col = 16 * (grp & 1) + 4 * (gi & 3);
            const uint32_t a = (uint32_t)(size_t)Vs + (uint32_t)(v_off(rbase, col >> 3) + (col & 7) * 2);
            vr[0][0][0] = ds_read_tr_asm_o<0>(a);
            vr[0][0][1] = ds_read_tr_asm_o<1024>(a);
            vr[1][0][0] = ds_read_tr_asm_o<2048>(a);
            vr[1][0][1] = ds_read_tr_asm_o<3072>(a);
        }
        __builtin_amdgcn_sched_barrier(0);
    } else {
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
    bm = xor32_max(bm);
    // Lazy rescale (T13): the running max m only moves when some query's tile max exceeds it by more than
    // 8 in the exp2 domain, so probabilities stay <= 2^8 (exact in fp32 accumulation, representable in bf16)
    // and the O / l rescale is skipped on almost every tile. The first tile always sets m (m = -inf).
    if (__builtin_expect(__any(bm > m + 8.0f / scale_log2), 0)) {   // loop-invariant threshold: 2 VALU, not 3
        const float mn = fmaxf(m, bm);
        const float alpha = __builtin_amdgcn_exp2f((m - mn) * scale_log2);
        m = mn;
        l *= alpha;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            o0[r] *= alpha;
            o1[r] *= alpha;
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
    if constexpr (ASM_TR) {
        static_assert(T == 1, "asm transposed-read path handles one 32-key tile");
        const int rbase = kb + 4 * (grp >> 1) + rq;
#pragma unroll
        for (int dt = PRE && VPF_ATTN_VEARLY ? 1 : 0; dt < 2; ++dt) {
            const int col = dt * 32 + 16 * (grp & 1) + 4 * cp;
            const int c16 = col >> 3, inner = (col & 7) * 2;
            const uint32_t a = (uint32_t)(size_t)Vs + (uint32_t)(v_off(rbase, c16) + inner);
            vr[0][dt][0] = ds_read_tr_asm_o<0>(a);
            vr[0][dt][1] = ds_read_tr_asm_o<1024>(a);
            vr[1][dt][0] = ds_read_tr_asm_o<2048>(a);
            vr[1][dt][1] = ds_read_tr_asm_o<3072>(a);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vr[0][0][0]), "+v"(vr[0][0][1]), "+v"(vr[0][1][0]), "+v"(vr[0][1][1]),
                     "+v"(vr[1][0][0]), "+v"(vr[1][0][1]), "+v"(vr[1][1][0]), "+v"(vr[1][1][1])::"memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
            for (int dt = 0; dt < 2; ++dt) {
                const bf16x4 lo = vr[st][dt][0], hi = vr[st][dt][1];
                const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                if (dt == 0) o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[0][st], o0, 0, 0, 0);
                else o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[0][st], o1, 0, 0, 0);
            }
        return;
    }
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

// The last key step when at most 8 keys of its 32 are real (N - kb <= 8: N = 197 -> 5 keys, N = 577 -> 1).
// Lane (l32, hh) holds key offsets (r & 3) + 8 (r >> 2) + 4 hh in s[r], so only r = 0..3 can be real: the
// max / exp / sum run on those 4 (12 of 16 registers are dead, and only their 4 need the key < N test),
// the probabilities of keys 8..31 are 0, and the second 16-key PV half (st = 1) is skipped. Padded K / V rows
// are copies of row N - 1 (finite), so the zero probabilities add exactly nothing, as in attn_step<MASK>.
__device__ __forceinline__ void attn_step_tail8(const char* Ks, const char* Vs, int kb, int N, int lane,
                                                const bf16x8 qf[4], float scale_log2, float& m, float& l,
                                                f32x16& o0, f32x16& o1) {
    // the lane id re-read through asm: its address math then stays inside this (last) step instead of being
    // hoisted above the key loop, where it held ~40 extra VGPRs and spilled
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
    const int l32 = lane & 31, hh = lane >> 5;
    f32x16 s = f32x16{};
    const int kr = kb + l32;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + k_off(kr, ks * 2 + hh));
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], s, 0, 0, 0);
    }
    float sv[4];
    float bm = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        sv[r] = kb + r + 4 * hh < N ? s[r] : -INFINITY;
        bm = fmaxf(bm, sv[r]);
    }
    bm = xor32_max(bm);
    if (__builtin_expect(__any(bm > m + 8.0f / scale_log2), 0)) {   // loop-invariant threshold: 2 VALU, not 3
        const float mn = fmaxf(m, bm);
        const float alpha = __builtin_amdgcn_exp2f((m - mn) * scale_log2);
        m = mn;
        l *= alpha;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            o0[r] *= alpha;
            o1[r] *= alpha;
        }
    }
    const float msc = m * scale_log2;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        sv[r] = __builtin_amdgcn_exp2f(fmaf(sv[r], scale_log2, -msc));
        l += sv[r];
    }
    const uint4 u = make_uint4(pack_bf2(sv[0], sv[1]), pack_bf2(sv[2], sv[3]), 0u, 0u);
    const bf16x8 pf = __builtin_bit_cast(bf16x8, u);
    const int grp = lane >> 4, gi = lane & 15;
    const int rq = gi >> 2, cp = gi & 3;
    bf16x4 vr[2][2];
    const int rbase = kb + 4 * (grp >> 1) + rq;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
        const int col = dt * 32 + 16 * (grp & 1) + 4 * cp;
        const int c16 = col >> 3, inner = (col & 7) * 2;
        const uint32_t a = (uint32_t)(size_t)Vs + (uint32_t)(v_off(rbase, c16) + inner);
        vr[dt][0] = ds_read_tr_asm_o<0>(a);
        vr[dt][1] = ds_read_tr_asm_o<1024>(a);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vr[0][0]), "+v"(vr[0][1]), "+v"(vr[1][0]), "+v"(vr[1][1])::"memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
        const bf16x4 lo = vr[dt][0], hi = vr[dt][1];
        const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        if (dt == 0) o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, o0, 0, 0, 0);
        else o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, o1, 0, 0, 0);
    }
}

// Software-pipelined form of the 32-query key step, split in two halves so that QK^T of chunk c + 1 is issued
// before the softmax of chunk c: its four MFMAs then run under that softmax's VALU instead of on the step's
// critical path (the step was QK^T -> wait -> max -> exp -> PV in one wave). Same operations in the same order per
// accumulator as attn_step<1, MASK, true, true> / attn_step_tail8: the results are bit-identical.
__device__ __forceinline__ int lane_id_opaque() {   // not hoistable: the address math stays in the step using it
    int lane;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
    return lane;
}
__device__ __forceinline__ f32x16 attn_qk32(const char* Ks, int kb, int lane, const bf16x8 qf[4]) {
    lane = lane_id_opaque();
    const int l32 = lane & 31, hh = lane >> 5;
    const int kr = kb + l32;
    bf16x8 kf[4];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) kf[ks] = *reinterpret_cast<const bf16x8*>(Ks + k_off(kr, ks * 2 + hh));
    f32x16 s = f32x16{};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[ks], qf[ks], s, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);   // issued here, ahead of the softmax that follows: they run under it
    return s;
}
// MODE 0: a full chunk; 1: the masked last chunk (keys >= N get probability 0); 2: the last chunk when at most 8 of
// its keys are real (attn_step_tail8's work: 4 live scores per lane, the second 16-key PV half skipped).
template <int MODE>
__device__ __forceinline__ void attn_sm_pv32(const char* Vs, int kb, int N, int lane, f32x16 s, float scale_log2,
                                             float& m, float& l, f32x16& o0, f32x16& o1) {
    lane = lane_id_opaque();
    const int hh = lane >> 5;
    constexpr int NR = MODE == 2 ? 4 : 16;
    float bm = -INFINITY;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        if constexpr (MODE != 0) {
            const int key = kb + (r & 3) + 8 * (r >> 2) + 4 * hh;
            if (key >= N) s[r] = -INFINITY;
        }
        bm = fmaxf(bm, s[r]);
    }
    bm = xor32_max(bm);
    if (__builtin_expect(__any(bm > m + 8.0f / scale_log2), 0)) {
        const float mn = fmaxf(m, bm);
        const float alpha = __builtin_amdgcn_exp2f((m - mn) * scale_log2);
        m = mn;
        l *= alpha;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            o0[r] *= alpha;
            o1[r] *= alpha;
        }
    }
    const float msc = m * scale_log2;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const float p = __builtin_amdgcn_exp2f(fmaf(s[r], scale_log2, -msc));
        s[r] = p;
        l += p;
    }
    bf16x8 pf[2];
    if constexpr (MODE == 2) {
        pf[0] = __builtin_bit_cast(bf16x8, make_uint4(pack_bf2(s[0], s[1]), pack_bf2(s[2], s[3]), 0u, 0u));
    } else {
#pragma unroll
        for (int st = 0; st < 2; ++st)
            pf[st] = __builtin_bit_cast(bf16x8, make_uint4(pack_bf2(s[8 * st + 0], s[8 * st + 1]),
                                                           pack_bf2(s[8 * st + 2], s[8 * st + 3]),
                                                           pack_bf2(s[8 * st + 4], s[8 * st + 5]),
                                                           pack_bf2(s[8 * st + 6], s[8 * st + 7])));
    }
    const int grp = lane >> 4, gi = lane & 15;
    const int rbase = kb + 4 * (grp >> 1) + (gi >> 2);
    constexpr int NST = MODE == 2 ? 1 : 2;
    bf16x4 vr[2][2][2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
        const int col = dt * 32 + 16 * (grp & 1) + 4 * (gi & 3);
        const uint32_t a = (uint32_t)(size_t)Vs + (uint32_t)(v_off(rbase, col >> 3) + (col & 7) * 2);
        vr[0][dt][0] = ds_read_tr_asm_o<0>(a);
        vr[0][dt][1] = ds_read_tr_asm_o<1024>(a);
        if constexpr (NST == 2) {
            vr[1][dt][0] = ds_read_tr_asm_o<2048>(a);
            vr[1][dt][1] = ds_read_tr_asm_o<3072>(a);
        }
    }
    if constexpr (NST == 2)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vr[0][0][0]), "+v"(vr[0][0][1]), "+v"(vr[0][1][0]), "+v"(vr[0][1][1]),
                     "+v"(vr[1][0][0]), "+v"(vr[1][0][1]), "+v"(vr[1][1][0]), "+v"(vr[1][1][1])::"memory");
    else
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vr[0][0][0]), "+v"(vr[0][0][1]), "+v"(vr[0][1][0]), "+v"(vr[0][1][1])
                     ::"memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int st = 0; st < NST; ++st)
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
            const bf16x4 lo = vr[st][dt][0], hi = vr[st][dt][1];
            const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            if (dt == 0) o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[st], o0, 0, 0, 0);
            else o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[st], o1, 0, 0, 0);
        }
}

// 16-query strip on v_mfma_f32_16x16x32_bf16: the last strip when it holds at most 16 real queries (N = 197 ->
// queries 192..207, 5 real), at half the MFMA and softmax work of a 32-query strip (which spent 27 of its 32 rows
// on padding). Operand maps of 16x16x32 (g = lane / 16): A lane = row lane % 16, K slots 8g .. 8g+7; B lane = column
// lane % 16, the same K slots; D lane = rows 4g .. 4g+3 of column lane % 16.
//   S^T = K Q^T per 16-key tile kt: A = K rows kb + 16 kt + lane % 16 (dims 32 kk + 8g ..), B = Q^T (query
//   q0 + lane % 16, dims 32 kk + 8g ..), so lane (query lane % 16, g) holds the scores of keys kb + 16 kt + 4g + r.
//   A query's row max / sum combine the 4 lanes lane % 16 + 16g (permlane16 + permlane32 swaps).
//   O^T += V^T P^T with the PV K slots permuted: slot 8g + 4 kt + r <-> key kb + 16 kt + 4g + r. The lane's own
//   8 probabilities are then its B fragment as they stand, and its V^T A fragment is two transposed reads: lane
//   16g + 4q + p supplies row kb + 4g + q (then + 16 rows = + 2048 B: the V swizzle keeps bit 1 of the row), dims
//   16 dt + 4p .. +3, and receives dim 16 dt + lane % 16 of those 4 keys (cdna_hip_programming.md T10).
//   O^T lane = dims 16 dt + 4g .. +3 of query lane % 16.
// MASK: keys >= N get probability 0 (the padded K / V rows are finite copies of row N - 1).
__device__ __forceinline__ float xor16_max(float x) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    float y;   // scores are never NaN: one v_max_f32 (as xor32_max)
    asm("v_max_f32 %0, %1, %2" : "=v"(y) : "v"(__uint_as_float(r[0])), "v"(__uint_as_float(r[1])));
    return y;
}
__device__ __forceinline__ float xor16_sum(float x) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool MASK>
__device__ __forceinline__ void attn_step16(const char* Ks, const char* Vs, int kb, int N, int lane, const bf16x8 qf[2],
                                            float scale_log2, float& m, float& l, f32x4 (&o)[4]) {
    const int r16 = lane & 15, g = lane >> 4;
    f32x4 s[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
        s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int kr = kb + 16 * kt + r16;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + k_off(kr, 4 * kk + g));
            s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[kk], s[kt], 0, 0, 0);
        }
    }
    float bm = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if constexpr (MASK) {
                if (kb + 16 * kt + 4 * g + r >= N) s[kt][r] = -INFINITY;
            }
            bm = fmaxf(bm, s[kt][r]);
        }
    bm = xor32_max(xor16_max(bm));
    if (__builtin_expect(__any(bm > m + 8.0f / scale_log2), 0)) {   // lazy rescale, as attn_step
        const float mn = fmaxf(m, bm);
        const float alpha = __builtin_amdgcn_exp2f((m - mn) * scale_log2);
        m = mn;
        l *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int r = 0; r < 4; ++r) o[dt][r] *= alpha;
    }
    const float msc = m * scale_log2;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float p = __builtin_amdgcn_exp2f(fmaf(s[kt][r], scale_log2, -msc));
            s[kt][r] = p;
            l += p;
        }
    const uint4 u = make_uint4(pack_bf2(s[0][0], s[0][1]), pack_bf2(s[0][2], s[0][3]), pack_bf2(s[1][0], s[1][1]),
                               pack_bf2(s[1][2], s[1][3]));
    const bf16x8 pf = __builtin_bit_cast(bf16x8, u);
    const int q = r16 >> 2, p4 = r16 & 3;
    bf16x4 vr[4][2];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
        const int c16 = 2 * dt + (p4 >> 1), inner = 8 * (p4 & 1);
        const uint32_t a = (uint32_t)(size_t)Vs + (uint32_t)(v_off(kb + 4 * g + q, c16) + inner);
        vr[dt][0] = ds_read_tr_asm_o<0>(a);
        vr[dt][1] = ds_read_tr_asm_o<2048>(a);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vr[0][0]), "+v"(vr[0][1]), "+v"(vr[1][0]), "+v"(vr[1][1]),
                 "+v"(vr[2][0]), "+v"(vr[2][1]), "+v"(vr[3][0]), "+v"(vr[3][1])::"memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
        const bf16x4 lo = vr[dt][0], hi = vr[dt][1];
        const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, o[dt], 0, 0, 0);
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

    // K/V staging: every DMA piece (8 rows x 128 B per wave-instruction, swizzle applied on the source
    // address, lane-linear LDS destination) is in flight at once, and the first strip's Q loads are issued
    // under it. Rows >= N are filled from row N-1: finite values whose keys are masked (probability 0).
    {
        const int ninstr = NP >> 3, sub = lane >> 3, slot = lane & 7;
        for (int j = wid; j < 2 * ninstr; j += nw) {
            const bool isv = j >= ninstr;
            const int g = isv ? j - ninstr : j;
            const int r = 8 * g + sub;
            const int c = isv ? (slot ^ (((r >> 1) & 1) << 2)) : (slot ^ ((r >> 1) & 7));
            const bf16_t* src = (isv ? vbase : kbase) + (int64_t)min(r, N - 1) * 3 * D + c * 8;
            __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)((isv ? Vs : Ks) + g * 1024), 16, 0, 0);
        }
    }
    const int l32 = lane & 31, hh = lane >> 5;
    const int nstrips = (q_rows + 31) >> 5;
    bf16x8 q0[4];
    {
        const int q = min(wid * 32 + l32, N - 1);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) q0[ks] = *reinterpret_cast<const bf16x8*>(qbase + (int64_t)q * 3 * D + ks * 16 + hh * 8);
    }
    __syncthreads();

    for (int strip = wid; strip < nstrips; strip += nw) {
        const int q = strip * 32 + l32;
        bf16x8 qf[4];
        if (strip == wid) {
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) qf[ks] = q0[ks];
        } else {
#pragma unroll
            for (int ks = 0; ks < 4; ++ks)
                qf[ks] = *reinterpret_cast<const bf16x8*>(qbase + (int64_t)min(q, N - 1) * 3 * D + ks * 16 + hh * 8);
        }
        f32x16 o0 = {}, o1 = {};
        float m = -INFINITY, l = 0.f;
        // full 32-key tiles need no mask; only the tail tile (NP - N padded keys) is masked. One S tile live
        // keeps the kernel at <= 128 VGPRs = 4 waves/SIMD (two 7-wave workgroups per CU).
        const int nfull = N & ~31;
        int kb = 0;
        for (; kb < nfull; kb += 32) attn_step<1, false>(Ks, Vs, kb, N, lane, qf, scale_log2, m, l, o0, o1);
        if (kb < NP) attn_step<1, true>(Ks, Vs, kb, N, lane, qf, scale_log2, m, l, o0, o1);
        l = xor32_sum(l);
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


// s_waitcnt vmcnt(n) for a runtime n (the immediate must be a constant): n >= the outstanding count is a no-op
__device__ __forceinline__ void wait_vmcnt(int n) {
    switch (n) {
#define VPF_VMW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
        VPF_VMW(1) VPF_VMW(2) VPF_VMW(3) VPF_VMW(4) VPF_VMW(5) VPF_VMW(6) VPF_VMW(7) VPF_VMW(8) VPF_VMW(9)
        VPF_VMW(10) VPF_VMW(11) VPF_VMW(12) VPF_VMW(13) VPF_VMW(14) VPF_VMW(15) VPF_VMW(16) VPF_VMW(17)
        VPF_VMW(18) VPF_VMW(19) VPF_VMW(20) VPF_VMW(21) VPF_VMW(22) VPF_VMW(23)
#undef VPF_VMW
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

// Key-pipelined variant: one 512-thread workgroup per (particle, head) as above, but the K/V images land in
// 32-key chunks and compute follows them: every wave issues its Q loads, then exactly one DMA piece per
// chunk (waves 0-3: the chunk's four 8-row K pieces, waves 4-7: its four V pieces), in chunk order. Before
// key tiles c .. c+CPB-1: a counted vmcnt (this wave's pieces of those chunks landed; later chunks stay in
// flight) and one s_barrier (everyone's did), so the QK^T / softmax / PV of the first tiles overlap the
// HBM fetch of the later ones instead of waiting for the whole 57 KiB image. Waves without a query strip
// (8 waves, 7 strips at N = 197) only move data and keep the barrier count. N <= 256 (one strip per wave).
// CPB: 32-key chunks per counted wait + barrier. Waiting for 4 chunks at a time (2 barriers at N = 197)
// measured 3-4 % faster than per-chunk barriers (1, 2, 3, 4: 1.223 / 1.210 / 1.196 / 1.178 ms at 4096 x 12
// heads, profiles/r1_gemm_lab/attn_cpb.txt): each barrier puts all 8 waves back in lockstep. Round 2 on the current
// kernel (profiles/r2_gemm_lab/attn_cpb_r2s5.txt, per-launch averages from bench.py): CPB 3 / 4 / 5 / 6 / 7 =
// 1.084 / 1.075 / 1.069 / 1.064 / 1.156 ms at N = 197; 6 and 4 are level on ViT-L (N = 577) and on the MX8 output.
#ifndef VPF_ATTN_CPB
#define VPF_ATTN_CPB 6   // -DVPF_ATTN_CPB=n builds A/B variants (tools/ab_libs.sh)
#endif
constexpr int PIPE_CPB = VPF_ATTN_CPB;
// OUT8: the output is written as MX8 (the fp8 path's proj A operand) instead of bf16: the same packed bf16
// values, quantised per 32-dim block (a block = 16 dims of a lane + 16 of its partner half-wave lane).
// TAIL16: when the last strip holds at most 16 real queries (q_rows % 32 in 1..16: N = 197), its wave runs the
// 16-query step (attn_step16) instead of a 32-query strip. That wave runs the same chunk loop (run_strip below, one
// template for both strip kinds), so every wave of the workgroup passes the same barriers at the same chunks: a wave
// whose loop took another barrier schedule would release its partners' reads of K / V chunks that have not landed
// (the round-2 attempt at this tail, which gave its 16-query wave a chunk loop of its own, read such chunks: NaNs
// on the 32-query strips).
// LAB (lab builds only, VPF_ATTN_LAB): 1 = no Q loads and no K / V DMA (compute on whatever LDS holds: the compute-only
// time), 2 = loads and barriers only (no key steps: the load-only time), 3 = staggered start (VPF_ATTN_STAGGER),
// 5 (VPF_ATTN_LAB=4) = the full kernel with the round-2 step order (attn_step without PRE).
template <int CPB, bool OUT8 = false, bool TAIL8 = true, bool TAIL16 = true, int LAB = 0>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void k_attn_bf16_pipe(
    const bf16_t* __restrict__ qkv, bf16_t* __restrict__ out, int N, int H, float scale_log2, int q_rows,
    uint8_t* __restrict__ out8 = nullptr, int ld8 = 0, uint8_t* __restrict__ s8 = nullptr, int lds8 = 0) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int NP = (N + 31) & ~31;
    const int NT = NP >> 5;              // 32-key chunks
    char* Ks = smem;
    char* Vs = smem + NP * ROWB;
    // LAB 7 (round 4 s2): persistent (gridDim = 2 x CUs, workgroup w takes units w, w + G, ..., lds8 = B H units), and
    // the second workgroup to start on each CU (a per-CU ticket from HW_ID / XCC_ID, s8 = zeroed int tickets) sleeps ld8
    // x ~8k cycles once, so the two resident workgroups run their load and compute phases half a unit apart for good
    auto unit = [&](const int bh) {
        const int b = bh / H, h = bh - (bh / H) * H;
        const int D = H * HD;
        const int64_t row0 = (int64_t)b * N;
        const bf16_t* qbase = qkv + row0 * 3 * D + h * HD;
        // LAB 7: the lane id re-read through an opaque asm per unit, so nothing lane-derived is hoisted out of the unit
        // loop (hoisted, it spilled 48 VGPRs)
        int lane_id = (int)(threadIdx.x & 63);
        if constexpr (LAB == 7) asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane_id));
        const int tid = (int)(threadIdx.x & ~63u) + lane_id, lane = lane_id;
        const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
        const int l32 = lane & 31, hh = lane >> 5;
        const int nstrips = (q_rows + 31) >> 5;
        // wave-uniform: this wave's strip holds query N - 1 and at most 16 real queries. Decided by N, not q_rows, so a
        // row's result does not depend on how many rows the call computes.
        const int nlast = (N - 1) >> 5;
        const bool w16 = TAIL16 && !OUT8 && wid == nlast && wid < nstrips && N - 32 * nlast <= 16;
    
        if constexpr (LAB == 3) {   // lab: the second resident workgroup of each CU starts ld8 x ~4k cycles late
            if (bh >= 256 && bh < 512)
                for (int i = 0; i < ld8; ++i) __builtin_amdgcn_s_sleep(64);
        }
        const int q = wid * 32 + l32;
        // Q fragments by inline-asm loads: hipcc does not count them, so it cannot merge them into a vmcnt(0) at
        // the first MFMA (which would also drain every K/V chunk). They are older than all DMA pieces, so the
        // first chunk's counted wait retires them; the empty asm after it pins every use below that wait.
        // 16-query strip: qf[kk] (kk < 2) = Q[32 wid + lane % 16][32 kk + 8 (lane / 16) ..] (attn_step16's B operand;
        // qf[2], qf[3] re-read the same bytes and are unused).
        // One asm load statement per register for both strip kinds, with the strip kind in the address only: loads issued
        // in two branches would leave each qf a phi of two asm outputs, and the copies that resolve it run at the branch
        // merge, before the loads land, so the registers the MFMAs read were stale (the NaNs of round 2's 16-query tail,
        // on the 32-query strips too).
        bf16x8 qf[4];
        {
            const bf16_t* qp = w16 ? qbase + (int64_t)min(wid * 32 + (lane & 15), N - 1) * 3 * D + 8 * (lane >> 4)
                                   : qbase + (int64_t)min(q, N - 1) * 3 * D + hh * 8;
            const int step = w16 ? 32 : 16;
            if constexpr (LAB == 1) {
    #pragma unroll
                for (int ks = 0; ks < 4; ++ks) qf[ks] = bf16x8{(short)(lane + ks), 0x3c00, 0x3c00, 0x3c00, 0, 0, 0, (short)wid};
            } else {
    #pragma unroll
            for (int ks = 0; ks < 4; ++ks)
                asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qf[ks]) : "v"(qp + (w16 ? (ks & 1) : ks) * step));
            }
        }
        if constexpr (LAB != 1) {
            const bool isv = wid >= 4;
            const int sub = lane >> 3, slot = lane & 7;
            const bf16_t* src0 = qbase + (isv ? 2 * D : D);
            char* img = isv ? Vs : Ks;
            for (int c = 0; c < NT; ++c) {
                const int g = c * 4 + (wid & 3);                 // 8-row piece index inside the image
                const int r = 8 * g + sub;
                const int ch = isv ? (slot ^ (((r >> 1) & 1) << 2)) : (slot ^ ((r >> 1) & 7));
                __builtin_amdgcn_global_load_lds((gptr_t)(src0 + (int64_t)min(r, N - 1) * 3 * D + ch * 8),
                                                 (lptr_t)(img + g * 1024), 16, 0, 0);
            }
        }
        // The Q loads are older than this wave's NT DMA pieces: landed once at most NT are outstanding. Wait and pin the
        // registers HERE, before the strip-kind branch: the compiler copies asm-load destinations wherever register
        // allocation wants (the phi / live-range copies of the w16 branch below moved qf before any wait, reading stale
        // registers: the round-2 NaN). The first chunk barrier waits for CPB chunks, so this costs nothing.
        wait_vmcnt(NT);
        asm volatile("" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]) :: "memory");
        const bool active = LAB != 2 && wid < nstrips;
        constexpr bool SWP = LAB == 6;   // lab: the software-pipelined 32-query strip (VPF_ATTN_LAB=5)
        const int nfull = N >> 5;             // chunks without padded keys
        // The chunk loop, one template for both strip kinds: the barrier schedule (a counted wait + s_barrier before
        // chunks 0, CPB, 2 CPB, ..., and before the padded tail chunk) depends on N and CPB only.
        auto run_strip = [&](auto k16, f32x16& o0, f32x16& o1, f32x4 (&o16)[4], float& m, float& l) {
            constexpr bool W16 = decltype(k16)::value;
            auto pin_q = [&]() {
                if constexpr (W16) asm volatile("" : "+v"(qf[0]), "+v"(qf[1]) :: "memory");
                else asm volatile("" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]) :: "memory");
            };
            if constexpr (!W16 && SWP) {
                // software-pipelined 32-query strip: the barrier before chunk group g (chunks g CPB ..) is taken before
                // QK^T of chunk g CPB, i.e. in iteration g CPB - 1; the same barriers in the same order as below
                if (!active) {   // a wave without a strip passes the same barriers
                    for (int c = 0; c < NT; c += CPB) {
                        wait_vmcnt(max(NT - c - CPB, 0));
                        __builtin_amdgcn_s_barrier();
                    }
                    return;
                }
                wait_vmcnt(max(NT - CPB, 0));
                __builtin_amdgcn_s_barrier();
                pin_q();
                // full chunks c < nfull; the tail chunk (c = nfull < NT) is peeled. (Unrolled by two, to alternate the
                // score tiles without the 8 v_mov_b64 of `cur = nxt`, hipcc spills 20-75 VGPRs at the 128 limit.)
                f32x16 cur = attn_qk32(Ks, 0, lane, qf);
                for (int c = 0; c < nfull; ++c) {
                    f32x16 nxt;
                    if (c + 1 < NT) {
                        if ((c + 1) % CPB == 0) {
                            wait_vmcnt(max(NT - (c + 1) - CPB, 0));
                            __builtin_amdgcn_s_barrier();
                            pin_q();
                        }
                        nxt = attn_qk32(Ks, (c + 1) * 32, lane, qf);
                    }
                    attn_sm_pv32<0>(Vs, c * 32, N, lane, cur, scale_log2, m, l, o0, o1);
                    cur = nxt;
                }
                if (nfull < NT) {
                    if (TAIL8 && N - nfull * 32 <= 8) attn_sm_pv32<2>(Vs, nfull * 32, N, lane, cur, scale_log2, m, l, o0, o1);
                    else attn_sm_pv32<1>(Vs, nfull * 32, N, lane, cur, scale_log2, m, l, o0, o1);
                }
                return;
            }
            int c = 0;
            for (; c < nfull; ++c) {
                if (c % CPB == 0) {   // chunks c .. c+CPB-1 landed for every wave
                    wait_vmcnt(max(NT - c - CPB, 0));
                    __builtin_amdgcn_s_barrier();
                    pin_q();
                }
                if (active) {
                    if constexpr (W16) attn_step16<false>(Ks, Vs, c * 32, N, lane, qf, scale_log2, m, l, o16);
                    else attn_step<1, false, true, LAB != 5>(Ks, Vs, c * 32, N, lane, qf, scale_log2, m, l, o0, o1);
                }
            }
            if (c < NT) {
                if (c % CPB == 0) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __builtin_amdgcn_s_barrier();
                    pin_q();
                }
                if (active) {
                    if constexpr (W16) attn_step16<true>(Ks, Vs, c * 32, N, lane, qf, scale_log2, m, l, o16);
                    else if (TAIL8 && N - c * 32 <= 8) attn_step_tail8(Ks, Vs, c * 32, N, lane, qf, scale_log2, m, l, o0, o1);
                    else attn_step<1, true, true, LAB != 5>(Ks, Vs, c * 32, N, lane, qf, scale_log2, m, l, o0, o1);
                }
            }
        };
        float m = -INFINITY, l = 0.f;
        if (w16) {
            f32x16 o0 = {}, o1 = {};
            f32x4 o16[4] = {};
            run_strip(std::true_type{}, o0, o1, o16, m, l);
            // the 4 lanes lane % 16 + 16 g share query 32 wid + lane % 16; lane holds dims 16 dt + 4g .. +3
            l = xor32_sum(xor16_sum(l));
            const float inv = 1.0f / l;
            const int qq = wid * 32 + (lane & 15);
            if (qq < q_rows) {
                bf16_t* orow = out + (row0 + qq) * D + h * HD + 4 * (lane >> 4);
    #pragma unroll
                for (int dt = 0; dt < 4; ++dt)
                    *reinterpret_cast<uint2*>(orow + 16 * dt) = make_uint2(pack_bf2(o16[dt][0] * inv, o16[dt][1] * inv),
                                                                          pack_bf2(o16[dt][2] * inv, o16[dt][3] * inv));
            }
            return;
        }
        f32x16 o0 = {}, o1 = {};
        f32x4 o16_unused[4];
        run_strip(std::false_type{}, o0, o1, o16_unused, m, l);
        if (!active) return;
        l = xor32_sum(l);
        const float inv = 1.0f / l;
        // Lane (l32, hh) holds dims 8k + 4hh .. +3 of query l32 for the eight 8-dim groups k (o0: k < 4, o1: k >= 4).
        // v_permlane32_swap per pair (k, k+1) gives the lower half-wave dims 8k..8k+7 and the upper half-wave
        // 8k+8..8k+15: one 16-B store per pair (cdna_hip_programming.md T21) instead of two 8-B stores.
        uint32_t gx[8], gy[8];
    #pragma unroll
        for (int k = 0; k < 8; ++k) {
            const f32x16& o = k < 4 ? o0 : o1;
            const int b4 = 4 * (k & 3);
            gx[k] = pack_bf2(o[b4] * inv, o[b4 + 1] * inv);
            gy[k] = pack_bf2(o[b4 + 2] * inv, o[b4 + 3] * inv);
        }
        uint4 ov[4];
    #pragma unroll
        for (int k = 0; k < 8; k += 2) {   // all lanes active: the swaps read the partner half-wave
            const auto rx = __builtin_amdgcn_permlane32_swap(gx[k], gx[k + 1], false, false);
            const auto ry = __builtin_amdgcn_permlane32_swap(gy[k], gy[k + 1], false, false);
            ov[k >> 1] = make_uint4(rx[0], ry[0], rx[1], ry[1]);
        }
        if constexpr (OUT8) {
            // lane (l32, hh) holds dims 16k + 8hh .. +7 (k = 0..3): block b = dims 32b .. 32b+31 is ov[2b], ov[2b+1]
            // of this lane and of its partner lane l32 + 32 (1 - hh)
            int E[2];
    #pragma unroll
            for (int b2 = 0; b2 < 2; ++b2) {
                uint32_t am = max(mx8_amax8(ov[2 * b2]), mx8_amax8(ov[2 * b2 + 1]));
                {
                    const auto r = __builtin_amdgcn_permlane32_swap(am, am, false, false);
                    am = max(r[0], r[1]);
                }
                E[b2] = mx8_block_exp(am);
            }
            if (q < q_rows) {
                const int64_t r = row0 + q;
                uint8_t* orow = out8 + r * ld8 + h * HD + 8 * hh;
    #pragma unroll
                for (int k = 0; k < 4; ++k) *reinterpret_cast<uint2*>(orow + 16 * k) = mx8_pack8(ov[k], E[k >> 1]);
                s8[mx8_scale_byte(r, h * HD + 32 * hh, lds8)] = (uint8_t)(E[hh] + 127);
            }
            return;
        }
        if (q < q_rows) {
            bf16_t* orow = out + (row0 + q) * D + h * HD + 8 * hh;
    #pragma unroll
            for (int k = 0; k < 4; ++k) *reinterpret_cast<uint4*>(orow + 16 * k) = ov[k];
        }
    };
    if constexpr (LAB == 7) {
        if (threadIdx.x == 0) {
            const uint32_t hw = __builtin_amdgcn_s_getreg(0xF804);    // HW_REG_HW_ID: cu 11:8, sh 12, se 15:13
            const uint32_t xcc = __builtin_amdgcn_s_getreg(0xF814);   // HW_REG_XCC_ID
            const int slot = (int)(((xcc & 7) << 8) | ((hw >> 8) & 0xFF));
            const int t = atomicAdd(reinterpret_cast<int*>(s8) + slot, 1);
            *reinterpret_cast<volatile int*>(smem) = t;
        }
        __syncthreads();
        const int ticket = *reinterpret_cast<volatile int*>(smem);
        __syncthreads();
        if (ticket & 1)
            for (int i = 0; i < ld8; ++i) __builtin_amdgcn_s_sleep(127);
        for (int u = blockIdx.x; u < lds8; u += gridDim.x) {
            unit(u);
            __builtin_amdgcn_s_waitcnt(0);   // this unit's stores / DMAs retired; every wave is done with the image
            __builtin_amdgcn_s_barrier();
        }
    } else {
        unit(blockIdx.x);
    }
}


// Persistent chunk-ring variant (round 4): the key-pipelined kernel's per-(particle, head) work, but a
// workgroup is resident for many (particle, head) units and the K / V chunks stream through a ring of R 32-key slots
// (8 KiB each: K rows | V rows, the same swizzled images as above at local row = key mod 32), so the DMA of the next
// unit's first chunks runs under the current unit's last key steps instead of each workgroup loading its whole image
// before it computes (the one-unit kernel's loads and compute overlapped only partly: 1.07 ms against 0.72 ms of loads
// and 0.84 ms of compute alone, profiles/r3_lab/attn_load_compute_split.txt).
//  * Grid: two 512-thread workgroups per CU (R x 8 KiB + 32 KiB of LDS each); workgroup w takes units w, w + G, ...
//  * Chunk stream: global chunk index g = j NT + c over this workgroup's units j and their chunks c; chunk g lives in
//    slot g % R. Every wave issues exactly one DMA piece per chunk (waves 0-3: the chunk's four 8-row K pieces, 4-7: its
//    V pieces), in g order; past the last chunk the pieces re-read the last chunk's rows into free slots (uniform
//    counts, bytes never read).
//  * Queries: each wave's 32-row query strip also arrives by LDS-DMA, into a 4 KiB area of its own (K-image layout),
//    one unit ahead: at unit j's start the wave reads Q(j) into registers and issues Q(j + 1)'s four pieces. (v1 loaded
//    Q into registers at each unit boundary; waiting for those loads retired every older ring piece too - in-order
//    vmcnt - so the ring drained at every unit: 1.54 ms against 1.06, profiles/r4_attn_ring_ab_v1.txt.)
//  * Groups of CB chunks: at the top of group s a counted vmcnt (this wave's pieces of chunks up to s CB + CB - 1
//    landed) and one s_barrier (everyone's pieces landed, and everyone is done with group s - 1), then the refill of the
//    group s - 1 slots with chunks s CB + R - CB .. s CB + R - 1. Every wait count is a closed form of (s or j, NT, R,
//    CB, the wave's store count) checked against a simulation of the issue sequence (tools/sim/attn_ring_counts.py).
//  * Per query row the arithmetic is the one-unit kernel's (same step functions, same order): bit-identical output.
// N <= 256 (one strip per wave), bf16 output.
// LABR (round 4 split of the ring's time): 1 = loads, waits and barriers only (no key steps), 2 = compute only (no K / V
// DMA: the steps read whatever the ring holds; the counted waits then retire nothing but Q)
template <int CB, int R, int LABR = 0>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void k_attn_bf16_ring(
    const bf16_t* __restrict__ qkv, bf16_t* __restrict__ out, int N, int H, int BH, float scale_log2, int q_rows) {
    static_assert(R >= 2 * CB, "the ring holds the group being computed and the group in flight");
    __shared__ __attribute__((aligned(16))) char ring[R * 8192 + 8 * 4096];
    const int NP = (N + 31) & ~31;
    const int NT = NP >> 5;
    const int D = H * HD;
    const int tid = threadIdx.x;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nstrips = (q_rows + 31) >> 5;
    const int nlast = (N - 1) >> 5;
    const bool w16 = wid == nlast && wid < nstrips && N - 32 * nlast <= 16;
    const bool active = wid < nstrips;
    const int S = active ? 4 : 0;          // output store instructions per unit of this wave
    const int G = gridDim.x;
    const int J = ((int)blockIdx.x < BH) ? (BH - 1 - (int)blockIdx.x) / G + 1 : 0;   // units of this workgroup
    if (J == 0) return;                    // workgroup-uniform
    const int Gtot = J * NT;
    const int nfull = N >> 5;
    char* qarea = ring + R * 8192 + wid * 4096;   // this wave's query strip (K-image layout, rows = strip rows)
    auto unit_base = [&](int j) -> const bf16_t* {
        const int bh = (int)blockIdx.x + j * G;
        const int b = bh / H, h = bh - (bh / H) * H;
        return qkv + (int64_t)b * N * 3 * D + h * HD;
    };
    // lane-derived addresses are recomputed where they are used (lane_id_opaque: not hoistable), so nothing of the
    // DMA / Q / store address math stays live across the key steps
    const bool isv = wid >= 4;
    auto issue = [&](int g) {   // this wave's piece of chunk g (clamped past the end) into slot g % R
        const int ln = lane_id_opaque();
        const int sub = ln >> 3, pslot = ln & 7;
        const int gc = min(g, Gtot - 1);
        const int j = gc / NT, c = gc - (gc / NT) * NT;
        const int rl = 8 * (wid & 3) + sub;            // local row in the chunk
        const int ch = isv ? (pslot ^ (((rl >> 1) & 1) << 2)) : (pslot ^ ((rl >> 1) & 7));
        const bf16_t* src = unit_base(j) + (isv ? 2 * D : D) + (int64_t)min(c * 32 + rl, N - 1) * 3 * D + ch * 8;
        char* dst = ring + (g % R) * 8192 + (isv ? 4096 : 0) + (wid & 3) * 1024;
        if constexpr (LABR != 2) __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)dst, 16, 0, 0);
    };
    auto issue_q = [&](int j) {   // the four 8-row pieces of this wave's query strip of unit min(j, J - 1)
        const int ln = lane_id_opaque();
        const int sub = ln >> 3, pslot = ln & 7;
        const bf16_t* qb = unit_base(min(j, J - 1));
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int rl = 8 * i + sub;
            const int ch = pslot ^ ((rl >> 1) & 7);
            __builtin_amdgcn_global_load_lds((gptr_t)(qb + (int64_t)min(wid * 32 + rl, N - 1) * 3 * D + ch * 8),
                                             (lptr_t)(qarea + i * 1024), 16, 0, 0);
        }
    };
    // ops issued after the piece of chunk s CB + CB - 1, at group top s (tools/sim/attn_ring_counts.py k_gt)
    auto k_gt = [&](int s) {
        const int gl = s * CB + CB - 1;
        const int si = max(0, (gl - R + CB) / CB);
        const int a = si * CB, b = s * CB;
        const int nq = b > a ? (b - 1) / NT - (a == 0 ? -1 : (a - 1) / NT) : 0;   // unit starts in [a, b)
        const int ns = b / NT - a / NT;                                             // unit ends in (a, b]
        return (R - 2 * CB) + 4 * nq + S * ns;
    };
    // ops issued after the last Q(j) piece, at unit j's start (k_qw)
    auto k_qw = [&](int j) { return j == 0 ? R : CB * ((j * NT) / CB - ((j - 1) * NT) / CB) + S; };
    bf16x8 qf[4];
    auto run = [&](auto k16) {
        constexpr bool W16 = decltype(k16)::value;
        issue_q(0);
        for (int g = 0; g < R - CB; ++g) issue(g);
        f32x16 o0 = {}, o1 = {};
        f32x4 o16[4] = {};
        float m = -INFINITY, l = 0.f;
        for (int j = 0; j < J; ++j) {
            if constexpr (W16) {
#pragma unroll
                for (int dt = 0; dt < 4; ++dt) o16[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
            } else {
                o0 = f32x16{};
                o1 = f32x16{};
            }
            m = -INFINITY;
            l = 0.f;
            for (int c = 0; c < NT; ++c) {
                const int g = j * NT + c;
                if (g % CB == 0) {
                    wait_vmcnt(k_gt(g / CB));
                    __builtin_amdgcn_s_barrier();
                    asm volatile("" ::: "memory");
#pragma unroll
                    for (int i = 0; i < CB; ++i) issue(g + R - CB + i);   // into the slots of group s - 1
                }
                if (c == 0) {
                    // Q(j) from this wave's LDS area into registers, then Q(j + 1)'s DMA into the area (after the reads
                    // have completed: lgkmcnt(0))
                    wait_vmcnt(k_qw(j));
                    asm volatile("" ::: "memory");
                    {
                        const int ln = lane_id_opaque();
                        if constexpr (W16) {
                            const int r16 = ln & 15, g4 = ln >> 4;
#pragma unroll
                            for (int kk = 0; kk < 4; ++kk)
                                qf[kk] = *reinterpret_cast<const bf16x8*>(qarea + k_off(r16, 4 * (kk & 1) + g4));
                        } else {
                            const int l32 = ln & 31, hh = ln >> 5;
#pragma unroll
                            for (int ks = 0; ks < 4; ++ks)
                                qf[ks] = *reinterpret_cast<const bf16x8*>(qarea + k_off(l32, ks * 2 + hh));
                        }
                    }
                    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3])::"memory");
                    issue_q(j + 1);
                }
                if (!active || LABR == 1) continue;
                // slot of chunk g, addressed with the global key base kb (the swizzles depend on key mod 32 only)
                const int kb = c * 32;
                const char* Ks = ring + (g % R) * 8192 - kb * ROWB;
                const char* Vs = Ks + 4096;
                // the lane id re-read per step: the steps' lane-derived LDS addresses are then computed in the step,
                // not hoisted out of both loops (which held ~10 VGPRs across them and spilled at the 128 limit)
                const int lane = lane_id_opaque();
                if (c < nfull) {
                    if constexpr (W16) attn_step16<false>(Ks, Vs, kb, N, lane, qf, scale_log2, m, l, o16);
                    else attn_step<1, false, true, true>(Ks, Vs, kb, N, lane, qf, scale_log2, m, l, o0, o1);
                } else {
                    if constexpr (W16) attn_step16<true>(Ks, Vs, kb, N, lane, qf, scale_log2, m, l, o16);
                    else if (N - kb <= 8) attn_step_tail8(Ks, Vs, kb, N, lane, qf, scale_log2, m, l, o0, o1);
                    else attn_step<1, true, true, true>(Ks, Vs, kb, N, lane, qf, scale_log2, m, l, o0, o1);
                }
            }
            // unit j's output rows (the pipe kernel's epilogues): S store instructions
            if (active) {
                const int ln = lane_id_opaque();
                const int bh = (int)blockIdx.x + j * G;
                const int b = bh / H, h = bh - (bh / H) * H;
                const int64_t row0 = (int64_t)b * N;
                if constexpr (W16) {
                    l = xor32_sum(xor16_sum(l));
                    const float inv = 1.0f / l;
                    const int qq = wid * 32 + (ln & 15);
                    bf16_t* orow = out + (row0 + min(qq, N - 1)) * D + h * HD + 4 * (ln >> 4);
                    if (qq < q_rows) {
#pragma unroll
                        for (int dt = 0; dt < 4; ++dt)
                            *reinterpret_cast<uint2*>(orow + 16 * dt) =
                                make_uint2(pack_bf2(o16[dt][0] * inv, o16[dt][1] * inv),
                                           pack_bf2(o16[dt][2] * inv, o16[dt][3] * inv));
                    }
                } else {
                    const int q = wid * 32 + (ln & 31), hh = ln >> 5;
                    l = xor32_sum(l);
                    const float inv = 1.0f / l;
                    uint32_t gx[8], gy[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const f32x16& o = k < 4 ? o0 : o1;
                        const int b4 = 4 * (k & 3);
                        gx[k] = pack_bf2(o[b4] * inv, o[b4 + 1] * inv);
                        gy[k] = pack_bf2(o[b4 + 2] * inv, o[b4 + 3] * inv);
                    }
                    uint4 ov[4];
#pragma unroll
                    for (int k = 0; k < 8; k += 2) {
                        const auto rx = __builtin_amdgcn_permlane32_swap(gx[k], gx[k + 1], false, false);
                        const auto ry = __builtin_amdgcn_permlane32_swap(gy[k], gy[k + 1], false, false);
                        ov[k >> 1] = make_uint4(rx[0], ry[0], rx[1], ry[1]);
                    }
                    bf16_t* orow = out + (row0 + min(q, N - 1)) * D + h * HD + 8 * hh;
                    if (q < q_rows) {
#pragma unroll
                        for (int k = 0; k < 4; ++k) *reinterpret_cast<uint4*>(orow + 16 * k) = ov[k];
                    }
                }
            }
        }
    };
    if (w16) run(std::true_type{});
    else run(std::false_type{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may outlive the workgroup
}

// CLS-only attention (q_rows == 1: the last encoder block, whose other query rows feed nothing): one wave
// per (particle, head), 4 per workgroup, no LDS, so occupancy is set by VGPRs and many heads stream K / V
// at once (the path is pure HBM streaming: 2 x N x 128 B per head for one query).
//   scores: lane j owns keys j, j+64, ...; K rows read whole (128 B) from global; fp32 dot with the CLS
//           query (broadcast loads), wave max / sum -> fp32 softmax in the exp2 domain;
//   PV:     lane (g, d8) = (lane >> 3, lane & 7) accumulates dims 8*d8..8*d8+7 over keys j = g (mod 8),
//           probabilities fetched with ds_bpermute, then a 3-step shuffle reduction over g.
constexpr int CLS_MAXT = 10;   // keys per lane in the score phase: N <= 640
__global__ __launch_bounds__(256) void k_attn_cls_bf16(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ out,
                                                       int N, int H, int BH, float scale_log2) {
    const int lane = threadIdx.x & 63;
    const int bh = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (bh >= BH) return;
    const int b = bh / H, h = bh - (bh / H) * H;
    const int D = H * HD;
    const bf16_t* base = qkv + (int64_t)b * N * 3 * D + h * HD;
    float q[HD];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const uint4 u = *reinterpret_cast<const uint4*>(base + c * 8);
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            q[c * 8 + 2 * e] = bf2f((bf16_t)(w[e] & 0xffff));
            q[c * 8 + 2 * e + 1] = bf2f((bf16_t)(w[e] >> 16));
        }
    }
    float sc[CLS_MAXT];
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < CLS_MAXT; ++t) {
        const int j = lane + 64 * t;
        float sv = -INFINITY;
        if (j < N) {
            const bf16_t* kr = base + (int64_t)j * 3 * D + D;
            float acc = 0.f;
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const uint4 u = *reinterpret_cast<const uint4*>(kr + c * 8);
                const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    acc = fmaf(q[c * 8 + 2 * e], bf2f((bf16_t)(w[e] & 0xffff)), acc);
                    acc = fmaf(q[c * 8 + 2 * e + 1], bf2f((bf16_t)(w[e] >> 16)), acc);
                }
            }
            sv = acc * scale_log2;
        }
        sc[t] = sv;
        mx = fmaxf(mx, sv);
    }
    mx = wave_max(mx);
    float l = 0.f;
#pragma unroll
    for (int t = 0; t < CLS_MAXT; ++t) {
        sc[t] = (lane + 64 * t < N) ? __builtin_amdgcn_exp2f(sc[t] - mx) : 0.f;
        l += sc[t];
    }
    l = wave_sum(l);
    const int g = lane >> 3, d8 = lane & 7;
    float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < CLS_MAXT; ++t) {
        if (64 * t >= N) break;
#pragma unroll
        for (int ii = 0; ii < 8; ++ii) {
            const int j = 64 * t + 8 * ii + g;            // keys of this (t, ii) block: 8 consecutive
            const float pj = __shfl(sc[t], 8 * ii + g, 64);
            if (j < N) {
                const uint4 u = *reinterpret_cast<const uint4*>(base + (int64_t)j * 3 * D + 2 * D + d8 * 8);
                const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    o[2 * e] = fmaf(pj, bf2f((bf16_t)(w[e] & 0xffff)), o[2 * e]);
                    o[2 * e + 1] = fmaf(pj, bf2f((bf16_t)(w[e] >> 16)), o[2 * e + 1]);
                }
            }
        }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        o[e] += __shfl_xor(o[e], 8, 64);
        o[e] += __shfl_xor(o[e], 16, 64);
        o[e] += __shfl_xor(o[e], 32, 64);
    }
    if (g == 0) {
        const float inv = 1.0f / l;
        bf16_t* orow = out + (int64_t)b * N * D + h * HD + d8 * 8;
        *reinterpret_cast<uint4*>(orow) = make_uint4(pack_bf2(o[0] * inv, o[1] * inv), pack_bf2(o[2] * inv, o[3] * inv),
                                                     pack_bf2(o[4] * inv, o[5] * inv), pack_bf2(o[6] * inv, o[7] * inv));
    }
}

// ---------------- fp32 parity path ----------------
// One thread per query; K / V of the (particle, head) stream through LDS in chunks of KC keys, so any N
// works (ViT-L/14 @ 336: N = 577). Exact two-pass softmax in key order: pass 1 the row max over all keys,
// pass 2 p = expf(s*scale - max), l += p, acc += p v.
constexpr int KC = 128;
__global__ __launch_bounds__(256) void k_attn_f32(const float* __restrict__ qkv, float* __restrict__ out, int N,
                                                  int H, float scale, int q_rows) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* Ks = reinterpret_cast<float*>(smem);
    float* Vs = Ks + KC * HD;
    const int bh = blockIdx.x;
    const int b = bh / H, h = bh - (bh / H) * H;
    const int D = H * HD;
    const int64_t row0 = (int64_t)b * N;
    const float* qbase = qkv + row0 * 3 * D + h * HD;
    auto stage = [&](int c0, bool with_v) {
        const int rows = min(KC, N - c0);
        __syncthreads();
        for (int idx = threadIdx.x; idx < rows * HD; idx += blockDim.x) {
            const int r = idx / HD, c = idx - (idx / HD) * HD;
            Ks[idx] = qbase[(int64_t)(c0 + r) * 3 * D + D + c];
            if (with_v) Vs[idx] = qbase[(int64_t)(c0 + r) * 3 * D + 2 * D + c];
        }
        __syncthreads();
        return rows;
    };
    for (int q0 = 0; q0 < q_rows; q0 += blockDim.x) {
        const int q = q0 + threadIdx.x;
        const bool active = q < q_rows;
        float qv[HD];
        for (int c = 0; c < HD; ++c) qv[c] = active ? qbase[(int64_t)q * 3 * D + c] : 0.f;
        float mx = -INFINITY;
        for (int c0 = 0; c0 < N; c0 += KC) {
            const int rows = stage(c0, false);
            if (active)
                for (int k = 0; k < rows; ++k) {
                    float s = 0.f;
                    for (int c = 0; c < HD; ++c) s = fmaf(qv[c], Ks[k * HD + c], s);
                    mx = fmaxf(mx, s * scale);
                }
        }
        float acc[HD];
        for (int c = 0; c < HD; ++c) acc[c] = 0.f;
        float l = 0.f;
        for (int c0 = 0; c0 < N; c0 += KC) {
            const int rows = stage(c0, true);
            if (active)
                for (int k = 0; k < rows; ++k) {
                    float s = 0.f;
                    for (int c = 0; c < HD; ++c) s = fmaf(qv[c], Ks[k * HD + c], s);
                    const float p = expf(s * scale - mx);
                    l += p;
                    for (int c = 0; c < HD; ++c) acc[c] = fmaf(p, Vs[k * HD + c], acc[c]);
                }
        }
        if (active) {
            float* orow = out + (row0 + q) * D + h * HD;
            for (int c = 0; c < HD; ++c) orow[c] = acc[c] / l;
        }
    }
}

}  // namespace

static int cu_count() {
    static int cached = 0;
    if (!cached) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
            cached = n;
        else
            cached = 256;
    }
    return cached;
}

static int attn_cus() {   // compute units of the current device (the persistent kernel's grid)
    static int cached = 0;
    if (!cached) {
        int dev = 0, n = 0;
        cached = (hipGetDevice(&dev) == hipSuccess &&
                  hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0) ? n : 256;
    }
    return cached;
}
// Attention kernel choice for N <= 256: 0 = k_attn_bf16_ring<2, 6>, 1 = the one-unit key-pipelined kernel, 2-3 = ring
// variants (CB, R) = (3, 6), (1, 6). Process state set by an explicit call (tests,
// A/B), never read from the environment.
static int g_attn_variant = 1;
VPF_API int vpf_attention_tune(int variant) {
    if (variant < 0 || variant > 5) return VPF_ERR_ARG;
    g_attn_variant = variant;
    return 0;
}

VPF_API int vpf_attention_bf16(const uint16_t* qkv, uint16_t* out, int64_t B, int N, int H, int hd, float scale,
                               int q_rows, void* stream) {
    if (B < 0 || N <= 0 || N > 640 || H <= 0 || hd != HD || B * H > INT32_MAX || q_rows < 1 || q_rows > N)
        return VPF_ERR_ARG;
    if (B == 0) return 0;
    const int NP = (N + 31) & ~31;
    size_t lds = (size_t)NP * ROWB * 2;
    const float scale_log2 = scale * 1.44269504088896341f;
    const int strips = (q_rows + 31) / 32;
    const int64_t BH = B * H;
    if (q_rows == 1) {
        hipLaunchKernelGGL(k_attn_cls_bf16, dim3((unsigned)((BH + 3) / 4)), dim3(256), 0, (hipStream_t)stream, qkv, out,
                           N, H, (int)BH, scale_log2);
        VPF_RETURN_LAUNCH();
    }
    if (N <= 256 && g_attn_variant != 1) {   // round 4: the persistent chunk-ring kernel (vpf_attention_tune 0 / 2 / 3)
        const int64_t BH = B * H;
        const unsigned G = (unsigned)std::min<int64_t>(BH, 2 * (int64_t)attn_cus());
        typedef void (*ring_fn)(const bf16_t*, bf16_t*, int, int, int, float, int);
        ring_fn fn = k_attn_bf16_ring<2, 6>;
        if (g_attn_variant == 2) fn = k_attn_bf16_ring<3, 6>;
        if (g_attn_variant == 4) fn = k_attn_bf16_ring<3, 6, 1>;
        if (g_attn_variant == 5) fn = k_attn_bf16_ring<3, 6, 2>;
        if (g_attn_variant == 3) fn = k_attn_bf16_ring<1, 6>;
        hipLaunchKernelGGL(fn, dim3(G), dim3(512), 0, (hipStream_t)stream, qkv, reinterpret_cast<bf16_t*>(out), N, H,
                           (int)BH, scale_log2, q_rows);
        VPF_RETURN_LAUNCH();
    }
    // N <= 256: the key-pipelined kernel (8 waves, one strip each). VPF_ATTN_MODE=0 selects the
    // whole-image kernel instead (A/B timing); N > 256 always takes it (waves loop over strips).
    const char* mode = getenv("VPF_ATTN_MODE");
    if (N <= 256 && !(mode && mode[0] == '0')) {
        // VPF_ATTN_TAIL=0: the general masked last step instead of attn_step_tail8; VPF_ATTN_TAIL16=0: the last
        // strip as a 32-query strip even when it holds <= 16 queries (A/B timing; every variant is tested)
        const char* tail = getenv("VPF_ATTN_TAIL");
        const char* t16 = getenv("VPF_ATTN_TAIL16");
        const bool tail8 = !(tail && tail[0] == '0'), tail16 = !(t16 && t16[0] == '0');
        typedef void (*pipe_fn)(const bf16_t*, bf16_t*, int, int, float, int, uint8_t*, int, uint8_t*, int);
        static const pipe_fn fns[4] = {k_attn_bf16_pipe<PIPE_CPB, false, false, false>,
                                       k_attn_bf16_pipe<PIPE_CPB, false, false, true>,
                                       k_attn_bf16_pipe<PIPE_CPB, false, true, false>,
                                       k_attn_bf16_pipe<PIPE_CPB, false, true, true>};
        static bool pipe_attr = false;   // benign race: idempotent attribute set
        if (!pipe_attr) {
            for (pipe_fn f : fns)
                (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            pipe_attr = true;
        }
        pipe_fn fn = fns[2 * tail8 + tail16];
        int lab_arg = 0;
#ifdef VPF_GEMM_LAB
        {   // lab builds: VPF_ATTN_LAB=1 compute only, =2 loads only (timing probes, outputs meaningless)
            static const pipe_fn lab[6] = {k_attn_bf16_pipe<PIPE_CPB, false, true, true, 1>,
                                           k_attn_bf16_pipe<PIPE_CPB, false, true, true, 2>,
                                           k_attn_bf16_pipe<PIPE_CPB, false, true, true, 3>,
                                           k_attn_bf16_pipe<PIPE_CPB, false, true, true, 5>,
                                           k_attn_bf16_pipe<PIPE_CPB, false, true, true, 6>,
                                           k_attn_bf16_pipe<PIPE_CPB, false, true, true, 7>};
            const char* le = getenv("VPF_ATTN_LAB");
            if (le && le[0] >= '1' && le[0] <= '6') {
                fn = lab[le[0] - '1'];
                (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            }
            const char* st = getenv("VPF_ATTN_STAGGER");   // LAB 3's / LAB 7's sleep count
            lab_arg = st ? atoi(st) : 0;
            if (le && le[0] == '6') {   // LAB 7: persistent grid of 2 workgroups per CU, per-CU tickets zeroed
                static int* tickets = nullptr;
                static int cus = 0;
                if (!tickets) {
                    if (hipMalloc((void**)&tickets, 2048 * sizeof(int)) != hipSuccess) return VPF_ERR_ARG;
                    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
                }
                (void)hipMemsetAsync(tickets, 0, 2048 * sizeof(int), (hipStream_t)stream);
                hipLaunchKernelGGL(fn, dim3((unsigned)(2 * cus)), dim3(512), lds, (hipStream_t)stream, qkv,
                                   reinterpret_cast<bf16_t*>(out), N, H, scale_log2, q_rows, (uint8_t*)nullptr, lab_arg,
                                   reinterpret_cast<uint8_t*>(tickets), (int)(B * H));
                VPF_RETURN_LAUNCH();
            }
            // round 4 s2: VPF_ATTN_LDS=<bytes> raises the dynamic LDS request (e.g. 100000: one workgroup per CU) to time
            // the kernel and its compute-only / load-only probes at one resident workgroup instead of two
            const char* lp = getenv("VPF_ATTN_LDS");
            if (lp && (size_t)atoi(lp) > lds) {
                lds = (size_t)atoi(lp);
                (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            }
        }
#endif
        hipLaunchKernelGGL(fn, dim3((unsigned)(B * H)), dim3(512), lds, (hipStream_t)stream, qkv,
                           reinterpret_cast<bf16_t*>(out), N, H, scale_log2, q_rows, (uint8_t*)nullptr, lab_arg,
                           (uint8_t*)nullptr, 0);
        VPF_RETURN_LAUNCH();
    }
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

VPF_API int vpf_attention_bf16_mx8(const uint16_t* qkv, int64_t B, int N, int H, int hd, float scale, uint8_t* out8,
                                   int64_t ld8, uint32_t* s8, int64_t lds, void* stream) {
    const int64_t D = (int64_t)H * HD;
    if (B < 0 || N <= 0 || N > 256 || H <= 0 || hd != HD || B * H > INT32_MAX || D % 128 != 0) return VPF_ERR_ARG;
    if (!qkv || !out8 || !s8 || ld8 < D || ld8 % 8 != 0 || ((uintptr_t)out8 & 7) || lds % 64 != 0 ||
        lds < B * N || ld8 > INT32_MAX || lds > INT32_MAX / 4)
        return VPF_ERR_ARG;
    if (B == 0) return 0;
    const int NP = (N + 31) & ~31;
    const size_t lds_bytes = (size_t)NP * ROWB * 2;
    static bool attr = false;   // benign race: idempotent attribute set
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_attn_bf16_pipe<PIPE_CPB, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL((k_attn_bf16_pipe<PIPE_CPB, true>), dim3((unsigned)(B * H)), dim3(512), lds_bytes,
                       (hipStream_t)stream, qkv, (bf16_t*)nullptr, N, H, scale * 1.44269504088896341f, N, out8, (int)ld8,
                       reinterpret_cast<uint8_t*>(s8), (int)lds);
    VPF_RETURN_LAUNCH();
}

VPF_API int vpf_attention_f32(const float* qkv, float* out, int64_t B, int N, int H, int hd, float scale,
                              int q_rows, void* stream) {
    if (B < 0 || N <= 0 || N > 4096 || H <= 0 || hd != HD || B * H > INT32_MAX || q_rows < 1 || q_rows > N)
        return VPF_ERR_ARG;
    if (B == 0) return 0;
    const size_t lds = (size_t)KC * HD * 4 * 2;   // one K chunk + one V chunk
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k_attn_f32, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    hipLaunchKernelGGL(k_attn_f32, dim3((unsigned)(B * H)), dim3(256), lds, (hipStream_t)stream, qkv, out, N, H,
                       scale, q_rows);
    VPF_RETURN_LAUNCH();
}
