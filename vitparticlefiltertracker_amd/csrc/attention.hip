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

// Kt / Vt: the tile's first K / V row in LDS; kb: its first key index (masking only).
template <bool MASK>
__device__ __forceinline__ void attn_step16(const char* Kt, const char* Vt, int kb, int N, int lane, const bf16x8 qf[2],
                                            float scale_log2, float& m, float& l, f32x4 (&o)[4]) {
    const int r16 = lane & 15, g = lane >> 4;
    f32x4 s[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
        s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int kr = 16 * kt + r16;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Kt + k_off(kr, 4 * kk + g));
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
        const uint32_t a = (uint32_t)(size_t)Vt + (uint32_t)(v_off(4 * g + q, c16) + inner);
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

// ---------------- round 5: the row sum on the matrix cores, and a speculative running max ----------------
// Per 32-key step a 32-query strip spent ~490 issue cycles per wave against 256 cycles of MFMA work (8 x 32x32x16):
// 16 v_exp_f32 (8 cyc each), 16 v_fma_f32 (the exp2 argument), 16 v_add_f32 (the row sum l), 8 v_max3_f32 + a permlane
// swap + compare (the running max), 8 v_cvt_pk_bf16_f32, address adds (MI355X_MICROARCH.md 'vector-instruction ISSUE
// cost'). Two of those groups move off the vector issue port here:
//  * l: each lane's bf16-packed probabilities (the PV MFMA's B operand) are summed by v_mfma_f32_4x4x4_16b_bf16 against
//    a ones A operand (four per step: 4 values per lane each, every accumulator register gets the lane's own sum), so
//    the 16 v_add_f32 become 4 MFMA issues. l is then the sum of the very bf16 weights the PV MFMA multiplies.
//  * the running max: the step exponentiates against the current m without looking for a new maximum, and the
//    accumulated l tells whether that was safe: a lane whose 16 probabilities sum to at most 2^8 has none above 2^8,
//    the bound the lazy rescale (T13) already allowed. Only when some lane's step sum exceeds it (or is not finite) does
//    the step recompute its scores, take the max, rescale O and l and exponentiate again (rare after the first keys).
//    The first key step of a strip takes the max as before (m = -inf).
__device__ __forceinline__ f32x4 lsum8(const bf16x8 p, f32x4 acc) {
    const bf16x4 ones = {(short)0x3F80, (short)0x3F80, (short)0x3F80, (short)0x3F80};
    const bf16x4 lo = __builtin_shufflevector(p, p, 0, 1, 2, 3);
    const bf16x4 hi = __builtin_shufflevector(p, p, 4, 5, 6, 7);
    acc = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(ones, lo, acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(ones, hi, acc, 0, 0, 0);
}

__device__ __forceinline__ float max16(const f32x16& s) {
    float bm = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) bm = fmaxf(bm, s[r]);
    return bm;
}

// S^T = K Q^T for one 32-key tile: the four K fragment reads together, then the four MFMAs (attn_step's PRE form)
// Kt: the tile's first K row in LDS (the swizzles depend on the row's low bits only, so a 32-row tile is addressed by
// its local rows)
__device__ __forceinline__ f32x16 qk32(const char* Kt, int lane, const bf16x8 qf[4]) {
    const int l32 = lane & 31, hh = lane >> 5;
    f32x16 s = f32x16{};
    bf16x8 kf[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) kf[ks] = *reinterpret_cast<const bf16x8*>(Kt + k_off(l32, ks * 2 + hh));
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[ks], qf[ks], s, 0, 0, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    __builtin_amdgcn_sched_barrier(0);
    return s;
}

// O^T += V^T P^T over one 32-key tile (both 16-key halves when HALVES == 2; the tail step's first half only when 1)
template <int HALVES>
__device__ __forceinline__ void pv32(const char* Vt, int lane, const bf16x8 pf[2], f32x16& o0, f32x16& o1) {
    const int grp = lane >> 4, gi = lane & 15;
    const int rq = gi >> 2, cp = gi & 3;
    const int rbase = 4 * (grp >> 1) + rq;
    bf16x4 vr[2][2][2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
        const int col = dt * 32 + 16 * (grp & 1) + 4 * cp;
        const int c16 = col >> 3, inner = (col & 7) * 2;
        const uint32_t a = (uint32_t)(size_t)Vt + (uint32_t)(v_off(rbase, c16) + inner);
        vr[0][dt][0] = ds_read_tr_asm_o<0>(a);
        vr[0][dt][1] = ds_read_tr_asm_o<1024>(a);
        if constexpr (HALVES == 2) {
            vr[1][dt][0] = ds_read_tr_asm_o<2048>(a);
            vr[1][dt][1] = ds_read_tr_asm_o<3072>(a);
        }
    }
    if constexpr (HALVES == 2)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vr[0][0][0]), "+v"(vr[0][0][1]), "+v"(vr[0][1][0]), "+v"(vr[0][1][1]),
                     "+v"(vr[1][0][0]), "+v"(vr[1][0][1]), "+v"(vr[1][1][0]), "+v"(vr[1][1][1])::"memory");
    else
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vr[0][0][0]), "+v"(vr[0][0][1]), "+v"(vr[0][1][0]), "+v"(vr[0][1][1])
                     ::"memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int st = 0; st < HALVES; ++st)
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
            const bf16x4 lo = vr[st][dt][0], hi = vr[st][dt][1];
            const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            if (dt == 0) o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[st], o0, 0, 0, 0);
            else o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[st], o1, 0, 0, 0);
        }
}

// The same step in the rounds 1-4 form (the N <= 256 kernel's): the row max of every tile (T13 lazy rescale when it
// moved by more than 2^8), l summed from the fp32 probabilities. Bit-identical to the rounds 1-4 attn_step.
template <bool MASK>
__device__ __forceinline__ void attn_step_pl(const char* Kt, const char* Vt, int kb, int N, int lane, const bf16x8 qf[4],
                                             float scale_log2, float& m, float& l, f32x16& o0, f32x16& o1) {
    const int hh = lane >> 5;
    f32x16 s = qk32(Kt, lane, qf);
    float bm = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        if constexpr (MASK) {
            if (kb + (r & 3) + 8 * (r >> 2) + 4 * hh >= N) s[r] = -INFINITY;
        }
        bm = fmaxf(bm, s[r]);
    }
    bm = xor32_max(bm);
    if (__builtin_expect(__any(bm > m + 8.0f / scale_log2), 0)) {   // loop-invariant threshold: 2 VALU, not 3
        const float mn = fmaxf(m, bm);
        const float alpha = __builtin_amdgcn_exp2f((m - mn) * scale_log2);
        m = mn;
        l *= alpha;
        o0 *= alpha;
        o1 *= alpha;
    }
    const float msc = m * scale_log2;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(fmaf(s[r], scale_log2, -msc));
        s[r] = p;
        l += p;
    }
    bf16x8 pf[2];
#pragma unroll
    for (int st = 0; st < 2; ++st)
        pf[st] = __builtin_bit_cast(bf16x8, make_uint4(pack_bf2(s[8 * st + 0], s[8 * st + 1]), pack_bf2(s[8 * st + 2], s[8 * st + 3]),
                                                       pack_bf2(s[8 * st + 4], s[8 * st + 5]), pack_bf2(s[8 * st + 6], s[8 * st + 7])));
    pv32<2>(Vt, lane, pf, o0, o1);
}

// attn_step_tail8 of rounds 1-4 (at most 8 real keys in the tile: s[0..3] only, the first 16-key PV half)
__device__ __forceinline__ void attn_step_tail8_pl(const char* Kt, const char* Vt, int kb, int N, int lane,
                                                   const bf16x8 qf[4], float scale_log2, float& m, float& l,
                                                   f32x16& o0, f32x16& o1) {
    // the lane id re-read through asm: its address math then stays inside this (last) step instead of being
    // hoisted above the key loop, where it held ~40 extra VGPRs and spilled
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
    const int hh = lane >> 5;
    const f32x16 s = qk32(Kt, lane, qf);
    float sv[4];
    float bm = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        sv[r] = kb + r + 4 * hh < N ? s[r] : -INFINITY;
        bm = fmaxf(bm, sv[r]);
    }
    bm = xor32_max(bm);
    if (__builtin_expect(__any(bm > m + 8.0f / scale_log2), 0)) {
        const float mn = fmaxf(m, bm);
        const float alpha = __builtin_amdgcn_exp2f((m - mn) * scale_log2);
        m = mn;
        l *= alpha;
        o0 *= alpha;
        o1 *= alpha;
    }
    const float msc = m * scale_log2;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        sv[r] = __builtin_amdgcn_exp2f(fmaf(sv[r], scale_log2, -msc));
        l += sv[r];
    }
    bf16x8 pf[2];
    pf[0] = __builtin_bit_cast(bf16x8, make_uint4(pack_bf2(sv[0], sv[1]), pack_bf2(sv[2], sv[3]), 0u, 0u));
    pf[1] = bf16x8{};
    pv32<1>(Vt, lane, pf, o0, o1);
}

// One 32-key step of a 32-query strip with l on the matrix cores and the speculative max (above). Kt / Vt: the tile's
// first K / V row in LDS; kb: its first key index (masking only). `first`: the strip's first key step (m = -inf: take
// the tile max). MASK: keys >= N in this tile get probability 0. lacc: the 4x4x4 MFMA accumulator (every register = the
// lane's running l).
template <bool MASK>
__device__ __forceinline__ void attn_step_lf(const char* Kt, const char* Vt, int kb, int N, int lane, const bf16x8 qf[4],
                                             float scale_log2, bool first, float& m, f32x4& lacc, f32x16& o0,
                                             f32x16& o1) {
    const int hh = lane >> 5;
    auto mask = [&](f32x16& t) {
        if constexpr (MASK) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (kb + (r & 3) + 8 * (r >> 2) + 4 * hh >= N) t[r] = -INFINITY;
        }
    };
    f32x16 s = qk32(Kt, lane, qf);
    mask(s);
    if (first) m = xor32_max(max16(s));
    bf16x8 pf[2];
    f32x4 ln;
    auto expo = [&](f32x16& t) {   // t: scores in, probabilities out
        const float msc = m * scale_log2;
#pragma unroll
        for (int r = 0; r < 16; ++r) t[r] = __builtin_amdgcn_exp2f(fmaf(t[r], scale_log2, -msc));
#pragma unroll
        for (int st = 0; st < 2; ++st)
            pf[st] = __builtin_bit_cast(bf16x8, make_uint4(pack_bf2(t[8 * st + 0], t[8 * st + 1]),
                                                           pack_bf2(t[8 * st + 2], t[8 * st + 3]),
                                                           pack_bf2(t[8 * st + 4], t[8 * st + 5]),
                                                           pack_bf2(t[8 * st + 6], t[8 * st + 7])));
        ln = lsum8(pf[1], lsum8(pf[0], lacc));
    };
    expo(s);
    if (!first && __builtin_expect(__any(!(ln[0] - lacc[0] <= 256.0f)), 0)) {
        f32x16 t = qk32(Kt, lane, qf);   // the scores again (s holds probabilities now)
        mask(t);
        const float mn = fmaxf(m, xor32_max(max16(t)));
        const float alpha = __builtin_amdgcn_exp2f((m - mn) * scale_log2);
        m = mn;
        lacc *= alpha;
        o0 *= alpha;
        o1 *= alpha;
        expo(t);
    }
    lacc = ln;
    pv32<2>(Vt, lane, pf, o0, o1);
}

// The last key step when at most 8 of its 32 keys are real (attn_step_tail8's register map: s[0..3] only), in the
// attn_step_lf form: one 4x4x4 MFMA for l, the speculative max, the first 16-key PV half.
__device__ __forceinline__ void attn_step_tail8_lf(const char* Kt, const char* Vt, int kb, int N, int lane,
                                                   const bf16x8 qf[4], float scale_log2, bool first, float& m,
                                                   f32x4& lacc, f32x16& o0, f32x16& o1) {
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
    const int hh = lane >> 5;
    const f32x16 s = qk32(Kt, lane, qf);
    float sv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) sv[r] = kb + r + 4 * hh < N ? s[r] : -INFINITY;
    auto max4 = [&]() { return xor32_max(fmaxf(fmaxf(sv[0], sv[1]), fmaxf(sv[2], sv[3]))); };
    if (first) m = max4();
    bf16x8 pf[2];
    pf[1] = bf16x8{};
    f32x4 ln;
    auto expo = [&]() {
        const float msc = m * scale_log2;
        float p[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) p[r] = __builtin_amdgcn_exp2f(fmaf(sv[r], scale_log2, -msc));
        pf[0] = __builtin_bit_cast(bf16x8, make_uint4(pack_bf2(p[0], p[1]), pack_bf2(p[2], p[3]), 0u, 0u));
        const bf16x4 ones = {(short)0x3F80, (short)0x3F80, (short)0x3F80, (short)0x3F80};
        ln = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(ones, __builtin_shufflevector(pf[0], pf[0], 0, 1, 2, 3), lacc, 0,
                                                    0, 0);
    };
    expo();
    if (!first && __builtin_expect(__any(!(ln[0] - lacc[0] <= 256.0f)), 0)) {
        const float mn = fmaxf(m, max4());
        const float alpha = __builtin_amdgcn_exp2f((m - mn) * scale_log2);
        m = mn;
        lacc *= alpha;
        o0 *= alpha;
        o1 *= alpha;
        expo();
    }
    lacc = ln;
    pv32<1>(Vt, lane, pf, o0, o1);
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
constexpr int PIPE_CPB = 6;
// OUT8: the output is written as MX8 (the fp8 path's proj A operand) instead of bf16: the same packed bf16
// values, quantised per 32-dim block (a block = 16 dims of a lane + 16 of its partner half-wave lane).
// TAIL16: when the last strip holds at most 16 real queries (q_rows % 32 in 1..16: N = 197), its wave runs the
// 16-query step (attn_step16) instead of a 32-query strip. That wave runs the same chunk loop (run_strip below, one
// template for both strip kinds), so every wave of the workgroup passes the same barriers at the same chunks: a wave
// whose loop took another barrier schedule would release its partners' reads of K / V chunks that have not landed
// (the round-2 attempt at this tail, which gave its 16-query wave a chunk loop of its own, read such chunks: NaNs
// on the 32-query strips).
// TAIL8: the last key step runs attn_step_tail8 when at most 8 of its keys are real.
// The round-3 lab variants of this kernel (compute-only / load-only probes, staggered start, software-pipelined strip,
// the round-2 step order) are in the lab build (tools/gemm_lab/attention_lab.hip).
template <int CPB, bool OUT8 = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void k_attn_bf16_pipe(
    const bf16_t* __restrict__ qkv, bf16_t* __restrict__ out, int N, int H, float scale_log2, int q_rows,
    uint8_t* __restrict__ out8 = nullptr, int ld8 = 0, uint8_t* __restrict__ s8 = nullptr, int lds8 = 0) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int NP = (N + 31) & ~31;
    const int NT = NP >> 5;              // 32-key chunks
    char* Ks = smem;
    char* Vs = smem + NP * ROWB;
    const int bh = blockIdx.x;
    const int b = bh / H, h = bh - (bh / H) * H;
    const int D = H * HD;
    const int64_t row0 = (int64_t)b * N;
    const bf16_t* qbase = qkv + row0 * 3 * D + h * HD;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l32 = lane & 31, hh = lane >> 5;
    const int nstrips = (q_rows + 31) >> 5;
    // sid: this wave's query strip (the identity; round 5 tried swapping waves 4, 5 with 6, 7 in every other workgroup so
    // that the half-work and idle strips of two co-resident workgroups land on different SIMDs: 1.4 % slower,
    // profiles/r5_lab/attn_simd_balance_ab.txt)
    const int sid = wid;
    // wave-uniform: this wave's strip holds query N - 1 and at most 16 real queries. Decided by N, not q_rows, so a
    // row's result does not depend on how many rows the call computes.
    const int nlast = (N - 1) >> 5;
    constexpr bool TAIL8 = true;
    const bool w16 = !OUT8 && sid == nlast && sid < nstrips && N - 32 * nlast <= 16;
    const int q = sid * 32 + l32;
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
        const bf16_t* qp = w16 ? qbase + (int64_t)min(sid * 32 + (lane & 15), N - 1) * 3 * D + 8 * (lane >> 4)
                               : qbase + (int64_t)min(q, N - 1) * 3 * D + hh * 8;
        const int step = w16 ? 32 : 16;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
            asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qf[ks]) : "v"(qp + (w16 ? (ks & 1) : ks) * step));
    }
    {
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
    // (Round 4: folding this wait and the pin into one asm statement per NT case, as ADVICE r3 suggested, made each qf a
    // phi of several asm outputs again and brought the NaNs back: profiles/r4_pytest_gpu_a.log. The rule kept: no branch
    // or merge between an asm load and the wait that retires it; the wait carries no register operands.)
    wait_vmcnt(NT);
    asm volatile("" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]) :: "memory");
    const bool active = sid < nstrips;
    const int nfull = N >> 5;             // chunks without padded keys
    // The chunk loop, one template for both strip kinds: the barrier schedule (a counted wait + s_barrier before
    // chunks 0, CPB, 2 CPB, ..., and before the padded tail chunk) depends on N and CPB only.
    auto run_strip = [&](auto k16, f32x16& o0, f32x16& o1, f32x4 (&o16)[4], float& m, float& l) {
        constexpr bool W16 = decltype(k16)::value;
        auto pin_q = [&]() {
            if constexpr (W16) asm volatile("" : "+v"(qf[0]), "+v"(qf[1]) :: "memory");
            else asm volatile("" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]) :: "memory");
        };
        int c = 0;
        for (; c < nfull; ++c) {
            if (c % CPB == 0) {   // chunks c .. c+CPB-1 landed for every wave
                wait_vmcnt(max(NT - c - CPB, 0));
                __builtin_amdgcn_s_barrier();
                pin_q();
            }
            if (active) {
                if constexpr (W16) attn_step16<false>(Ks + c * 4096, Vs + c * 4096, c * 32, N, lane, qf, scale_log2, m, l, o16);
                else attn_step_pl<false>(Ks + c * 4096, Vs + c * 4096, c * 32, N, lane, qf, scale_log2, m, l, o0, o1);
            }
        }
        if (c < NT) {
            if (c % CPB == 0) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                pin_q();
            }
            if (active) {
                if constexpr (W16) attn_step16<true>(Ks + c * 4096, Vs + c * 4096, c * 32, N, lane, qf, scale_log2, m, l, o16);
                else if (TAIL8 && N - c * 32 <= 8)
                    attn_step_tail8_pl(Ks + c * 4096, Vs + c * 4096, c * 32, N, lane, qf, scale_log2, m, l, o0, o1);
                else attn_step_pl<true>(Ks + c * 4096, Vs + c * 4096, c * 32, N, lane, qf, scale_log2, m, l, o0, o1);
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
        const int qq = sid * 32 + (lane & 15);
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
}


// ---------------- N > 256 (ViT-L/14 @ 336: N = 577): K / V streamed through a ring, queries in blocks ----------------
// The N <= 256 kernel keeps a head's whole K / V image in LDS (57 KiB at N = 197); at N = 577 that image is 152 KiB, so
// one workgroup fits a CU, its load phase is not overlapped, and 19 strips over 8 waves leave the SIMDs unbalanced
// (rounds 1-4: 9.93 ms per launch at 4096 x 16 heads = 0.225 of the bf16 peak). Here (rounds 5-6):
//  * one workgroup = 4 waves = one 128-query block of one (particle, head): QB = 5 blocks cover N = 577 (four blocks of
//    4 x 32-query strips, then 2 strips, and the 16-query strip of query 576 on a wave of its own, attn_step16). A
//    4-wave workgroup has one wave on each SIMD whatever the dispatcher does (6-wave workgroups land 2/4/3/3 per SIMD,
//    tools/micro/simd_probe.hip). The 16-query strip always has a wave of its own: the host adds a block when every
//    wave of the last one holds a 32-query strip (N % 32 in 1..16 with a multiple of 4 full strips, e.g. N = 400).
//  * four workgroups per CU (round 6; round 5 ran three): one wave of each on every SIMD, so <= 128 VGPRs. A wave runs
//    one strip kind (run_strip, instantiated per kind), so the 32-query strip's registers (o0 / o1 / lacc) and the
//    16-query strip's (o16) are never live together, and one Q load set serves both kinds; the steps are attn_step_lf
//    with the V^T reads after the softmax (126 VGPRs).
//  * K / V arrive in 32-key chunks (4 KiB of K + 4 KiB of V) through a ring of 4 chunk slots (32 KiB per workgroup). A
//    group of 2 chunks = 16 LDS-DMA pieces of 1 KiB, 4 per wave; two groups are resident: while one is computed, the
//    next is in flight. One counted vmcnt + s_barrier per group; after the barrier of group g every wave has finished
//    group g - 1, whose slots take group g + 1.
//  * the blocks of a unit run on one XCD (blockIdx b -> XCD b % 8; consecutive blocks of that XCD are one unit's blocks),
//    so four of the five K / V reads of a unit are L2 hits.
// A row's bits depend on N only, not on q_rows or on the block it falls in. The variants measured against this form
// (round 5: 6-wave / 3-chunk workgroups, the attn_step_pl steps, software pipelining, two strips per wave,
// profiles/r5_lab/attn_stream_*_ab.txt; round 6: ring depths, the step forms and the wave counts,
// profiles/r6_lab/attn_stream_occupancy_ab.txt, tools/variants/_attn_split.py) are not compiled here.
constexpr int STREAM_WAVES = 4;
constexpr int STREAM_CPB = 2;                      // 32-key chunks per group (8 pieces each: 4 per wave per group)
constexpr int STREAM_RING = 2;                     // groups resident in the ring
constexpr int STREAM_SLOTS = STREAM_CPB * STREAM_RING;

__global__ __launch_bounds__(STREAM_WAVES * 64) __attribute__((amdgpu_waves_per_eu(4))) void k_attn_stream(
    const bf16_t* __restrict__ qkv, bf16_t* __restrict__ out, int N, int H, float scale_log2, int q_rows, int QB,
    int BH) {
    constexpr int WAVES = STREAM_WAVES;
    constexpr int STREAM_LDS = STREAM_SLOTS * 2 * 4096;
    static_assert((STREAM_CPB * 8) % WAVES == 0, "a group's DMA pieces split evenly over the waves");
    constexpr int PPW = STREAM_CPB * 8 / WAVES;    // DMA pieces per wave per group
    __shared__ __attribute__((aligned(16))) char smem[STREAM_LDS];
    char* Ks = smem;
    char* Vs = smem + STREAM_SLOTS * 4096;
    const int xcd = blockIdx.x & 7, w8 = blockIdx.x >> 3;
    const int u = (w8 / QB) * 8 + xcd, qb = w8 - (w8 / QB) * QB;
    if (u >= BH) return;                           // padding of the XCD-grouped grid: the whole workgroup leaves
    const int b = u / H, h = u - (u / H) * H;
    const int D = H * HD;
    const int64_t row0 = (int64_t)b * N;
    const bf16_t* qbase = qkv + row0 * 3 * D + h * HD;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l32 = lane & 31, hh = lane >> 5;
    const int NT = (N + 31) >> 5;                  // 32-key chunks
    const int NG = (NT + STREAM_CPB - 1) / STREAM_CPB;
    const int SF = N >> 5, tail = N & 31;
    const int SF32 = SF + (tail > 16 ? 1 : 0);     // 32-query strips (the last one partial when tail > 16)
    const int st = qb * WAVES + wid;
    const bool act32 = st < SF32 && st * 32 < q_rows;
    const int idle0 = SF32 - (QB - 1) * WAVES;     // first wave of the last block without a 32-query strip
    const bool act16 = tail >= 1 && tail <= 16 && 32 * SF < q_rows && qb == QB - 1 && wid == idle0;   // host: idle0 < WAVES

    // Q fragments by inline-asm loads, one set for both strip kinds with the kind in the address only (k_attn_bf16_pipe's
    // rule: no branch or merge between an asm load and the wait that retires it). 16-query strip: qf[kk] (kk < 2) =
    // Q[32 SF + lane % 16][32 kk + 8 (lane / 16) ..] (attn_step16's B operand; qf[2], qf[3] re-read the same bytes).
    bf16x8 qf[4];
    {
        const bf16_t* qp = act16 ? qbase + (int64_t)min(SF * 32 + (lane & 15), N - 1) * 3 * D + 8 * (lane >> 4)
                                 : qbase + (int64_t)min(st * 32 + l32, N - 1) * 3 * D + hh * 8;
        const int step = act16 ? 32 : 16;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
            asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qf[ks]) : "v"(qp + (act16 ? (ks & 1) : ks) * step));
    }
    // group g = chunks [2g, 2g + 2): piece pi = 0..15 of a group is chunk pi / 8, K (pi & 4 == 0) or V, rows 8 (pi & 3) ..
    // + 7 of that chunk (one 1 KiB wave-instruction, lane-linear destination, swizzle on the source address as in
    // k_attn_bf16_pipe); wave w issues pieces w, w + WAVES, ... Rows >= N read row N - 1 (finite; masked keys).
    auto issue_group = [&](int g) {
        // the lane id re-read through asm: the pieces' addresses are then computed where they are issued instead of
        // being hoisted above the group loop as invariants (which spilled, and a scratch reload's vmcnt wait would
        // drain the DMA stream)
        int ln;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
        const int sub = ln >> 3, slot = ln & 7;
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
            const int pi = wid + WAVES * i;
            const int cc = pi >> 3, isv = (pi >> 2) & 1, j = pi & 3;
            const int c = g * STREAM_CPB + cc;
            const int r = c * 32 + 8 * j + sub;
            const int ch = isv ? (slot ^ (((r >> 1) & 1) << 2)) : (slot ^ ((r >> 1) & 7));
            const int sl = c % STREAM_SLOTS;
            __builtin_amdgcn_global_load_lds(
                (gptr_t)(qbase + (isv ? 2 * D : D) + (int64_t)min(r, N - 1) * 3 * D + ch * 8),
                (lptr_t)((isv ? Vs : Ks) + sl * 4096 + j * 1024), 16, 0, 0);
        }
    };
    const int g0 = min(NG, STREAM_RING);
    for (int g = 0; g < g0; ++g) issue_group(g);
    // the Q loads are older than every DMA piece: landed once at most PPW * g0 pieces are outstanding; wait and pin here
    wait_vmcnt(PPW * g0);
    asm volatile("" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]) :: "memory");
    const int nfull = N >> 5;                      // chunks without padded keys
    // the group loop and the stores of one strip kind; the barrier schedule depends on N only, so every wave of the
    // workgroup passes the same barriers whatever its kind (or none: act = false keeps the barriers, computes nothing)
    auto run_strip = [&](auto k16, bool act) {
        constexpr bool W16 = decltype(k16)::value;
        f32x16 o0 = {}, o1 = {};
        f32x4 lacc = {};
        f32x4 o16[4] = {};
        float m = -INFINITY, l = 0.f;
        auto pin_q = [&]() {
            if constexpr (W16) asm volatile("" : "+v"(qf[0]), "+v"(qf[1]) :: "memory");
            else asm volatile("" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]) :: "memory");
        };
        for (int g = 0; g < NG; ++g) {
            // this wave's pieces of group g have landed (the groups issued after it stay in flight), then every wave's
            const int issued = min(NG, max(STREAM_RING, g + STREAM_RING - 1));
            wait_vmcnt(PPW * (issued - g - 1));
            __builtin_amdgcn_s_barrier();
            pin_q();
            // into group g - 1's slots, which every wave has finished
            if (g >= 1 && g + STREAM_RING - 1 < NG) issue_group(g + STREAM_RING - 1);
            const int c_end = min((g + 1) * STREAM_CPB, nfull);
#pragma unroll 1
            for (int c = g * STREAM_CPB; c < c_end; ++c) {   // the group's chunks without padded keys
                const int sl = c % STREAM_SLOTS;
                const char* Kt = Ks + sl * 4096;
                const char* Vt = Vs + sl * 4096;
                if (act) {
                    if constexpr (W16) attn_step16<false>(Kt, Vt, c * 32, N, lane, qf, scale_log2, m, l, o16);
                    else attn_step_lf<false>(Kt, Vt, c * 32, N, lane, qf, scale_log2, c == 0, m, lacc, o0, o1);
                }
            }
        }
        if (nfull < NT && act) {   // the chunk with padded keys: the last one, in the last group (its barrier has passed)
            const int c = nfull, sl = c % STREAM_SLOTS;
            const char* Kt = Ks + sl * 4096;
            const char* Vt = Vs + sl * 4096;
            if constexpr (W16) attn_step16<true>(Kt, Vt, c * 32, N, lane, qf, scale_log2, m, l, o16);
            else if (N - c * 32 <= 8) attn_step_tail8_lf(Kt, Vt, c * 32, N, lane, qf, scale_log2, c == 0, m, lacc, o0, o1);
            else attn_step_lf<true>(Kt, Vt, c * 32, N, lane, qf, scale_log2, c == 0, m, lacc, o0, o1);
        }
        if (!act) return;
        if constexpr (W16) {   // the 4 lanes lane % 16 + 16 g share query 32 SF + lane % 16; lane: dims 16 dt + 4g .. +3
            const float inv = 1.0f / xor32_sum(xor16_sum(l));
            const int qq = SF * 32 + (lane & 15);
            if (qq < q_rows) {
                bf16_t* orow = out + (row0 + qq) * D + h * HD + 4 * (lane >> 4);
#pragma unroll
                for (int dt = 0; dt < 4; ++dt)
                    *reinterpret_cast<uint2*>(orow + 16 * dt) = make_uint2(pack_bf2(o16[dt][0] * inv, o16[dt][1] * inv),
                                                                          pack_bf2(o16[dt][2] * inv, o16[dt][3] * inv));
            }
        } else {
            const float inv = 1.0f / xor32_sum(lacc[0]);
            uint32_t gx[8], gy[8];   // as k_attn_bf16_pipe: permlane32 pairs -> one 16-B store per 8-dim pair
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const f32x16& o = k < 4 ? o0 : o1;
                const int b4 = 4 * (k & 3);
                gx[k] = pack_bf2(o[b4] * inv, o[b4 + 1] * inv);
                gy[k] = pack_bf2(o[b4 + 2] * inv, o[b4 + 3] * inv);
            }
            const int q = st * 32 + l32;
            uint4 ov[4];
#pragma unroll
            for (int k = 0; k < 8; k += 2) {
                const auto rx = __builtin_amdgcn_permlane32_swap(gx[k], gx[k + 1], false, false);
                const auto ry = __builtin_amdgcn_permlane32_swap(gy[k], gy[k + 1], false, false);
                ov[k >> 1] = make_uint4(rx[0], ry[0], rx[1], ry[1]);
            }
            if (q < q_rows) {
                bf16_t* orow = out + (row0 + q) * D + h * HD + 8 * hh;
#pragma unroll
                for (int k = 0; k < 4; ++k) *reinterpret_cast<uint4*>(orow + 16 * k) = ov[k];
            }
        }
    };
    if (act16) run_strip(std::true_type{}, true);
    else run_strip(std::false_type{}, act32);
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

VPF_API int vpf_attention_bf16(const uint16_t* qkv, uint16_t* out, int64_t B, int N, int H, int hd, float scale,
                               int q_rows, void* stream) {
    if (B < 0 || N <= 0 || N > 640 || H <= 0 || hd != HD || B * H > INT32_MAX || q_rows < 1 || q_rows > N)
        return VPF_ERR_ARG;
    if (B == 0) return 0;
    const int NP = (N + 31) & ~31;
    const size_t lds = (size_t)NP * ROWB * 2;
    const float scale_log2 = scale * 1.44269504088896341f;
    const int64_t BH = B * H;
    if (q_rows == 1) {
        hipLaunchKernelGGL(k_attn_cls_bf16, dim3((unsigned)((BH + 3) / 4)), dim3(256), 0, (hipStream_t)stream, qkv, out,
                           N, H, (int)BH, scale_log2);
        VPF_RETURN_LAUNCH();
    }
    // N <= 256: the key-pipelined kernel (8 waves, one strip each, the head's whole K / V image in LDS); N > 256: the
    // key-streamed, query-blocked kernel. (Round 4's persistent chunk-ring form of the N <= 256 kernel is bit-identical
    // but 1.5x slower: tools/gemm_lab/attention_lab.hip, profiles/r4_lab/attn_ring_ab_v*.txt.)
    if (N <= 256) {
        static bool pipe_attr = false;   // benign race: idempotent attribute set
        if (!pipe_attr) {
            (void)hipFuncSetAttribute((const void*)k_attn_bf16_pipe<PIPE_CPB, false>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            pipe_attr = true;
        }
        hipLaunchKernelGGL((k_attn_bf16_pipe<PIPE_CPB, false>), dim3((unsigned)(B * H)), dim3(512), lds,
                           (hipStream_t)stream, qkv, reinterpret_cast<bf16_t*>(out), N, H, scale_log2, q_rows,
                           (uint8_t*)nullptr, 0, (uint8_t*)nullptr, 0);
        VPF_RETURN_LAUNCH();
    }
    constexpr int W = STREAM_WAVES;
    const int sf32 = (N >> 5) + ((N & 31) > 16 ? 1 : 0);
    const int need = sf32 < (q_rows + 31) / 32 ? sf32 : (q_rows + 31) / 32;   // 32-query strips holding rows < q_rows
    const int t32 = N & 31;   // + the 16-query strip, which runs on a wave of its own (k_attn_stream's idle0 < WAVES)
    const int need16 = need + (t32 >= 1 && t32 <= 16 && 32 * (N >> 5) < q_rows ? 1 : 0);
    const int QB = need16 > W ? (need16 + W - 1) / W : 1;
    const int64_t blocks = (BH + 7) / 8 * 8 * QB;
    if (blocks > INT32_MAX) return VPF_ERR_ARG;
    hipLaunchKernelGGL(k_attn_stream, dim3((unsigned)blocks), dim3(64 * W), 0,
                       (hipStream_t)stream,
                       reinterpret_cast<const bf16_t*>(qkv), reinterpret_cast<bf16_t*>(out), N, H, scale_log2, q_rows,
                       QB, (int)BH);
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
