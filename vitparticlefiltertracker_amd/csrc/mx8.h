// MX-fp8 (OCP MX: e4m3fn elements, one e8m0 scale per 32 consecutive K values) device helpers shared by the
// GEMM epilogues (gemm_common.h), the quantiser (gemm_mx8.hip) and the attention output (attention.hip).
#pragma once
#include "vpf_common.h"

namespace vpf {

// ---------------- MX fp8 (OCP e4m3fn elements, e8m0 scale per 32 consecutive K values) ----------------
// Layout (vpf.h "MX8 operands"): elements X8[row][k] (1 B each, row stride ld8 bytes). Scales: per 128-deep
// K-tile t a plane of lds words (lds % 64 == 0), rows in bricks of 64: the scale of (row r, K-block
// kb = (k / 32) % 4) is byte (r / 16) % 4 of word t * lds + (r / 64) * 64 + kb * 16 + r % 16 (mx8_scale_byte).
// A 256-row tile's scales for one K-tile are one contiguous 1 KiB DMA, and a GEMM lane (row r16 + 16 f of a
// brick, K-block fq) finds the scales of the 4 fragments f = 0..3 it multiplies in the 4 bytes of ONE word,
// which v_mfma_scale's op_sel picks byte by byte (no shifts, 3 scale VGPRs per K-tile instead of 12).
__device__ __forceinline__ int64_t mx8_scale_byte(int64_t r, int k, int lds) {
    return ((int64_t)(k >> 7) * lds + (r >> 6) * 64 + ((k >> 5) & 3) * 16 + (r & 15)) * 4 + ((r >> 4) & 3);
}
//
// Block exponent: the smallest E with amax * 2^-E <= 448 (e4m3's largest finite value, 1.75 * 2^8), so no
// element saturates; e8m0 byte = E + 127, E clamped to [-127, 125]. Elements: RNE(x * 2^-E) (x * 2^-E is exact
// in fp32), one v_cvt_pk_fp8_f32 per pair. Dequantised value = e4m3(q) * 2^(byte - 127).
__device__ __forceinline__ int mx8_block_exp(uint32_t amax_bf16) {   // amax as |bf16| bits (sign clear)
    const uint32_t be = amax_bf16 >> 7;                                // biased exponent (0 = zero / subnormal)
    const int ex = be ? (int)be - 127 : -126;
    int E = ex - 8 + ((amax_bf16 & 0x7f) > 0x60 ? 1 : 0);             // mantissa > 1.75 needs one more
    return min(max(E, -127), 125);
}

// |x| max of 8 packed bf16 values, as |bf16| bits (integer order = magnitude order): sign bits cleared on both halves,
// packed 16-bit maxima (v_pk_max_u16), then the two halves (8 VALU instead of 13)
typedef unsigned short vpf_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t mx8_amax8(uint4 v) {
    const vpf_u16x2 a = __builtin_bit_cast(vpf_u16x2, v.x & 0x7fff7fffu), b = __builtin_bit_cast(vpf_u16x2, v.y & 0x7fff7fffu);
    const vpf_u16x2 c = __builtin_bit_cast(vpf_u16x2, v.z & 0x7fff7fffu), d = __builtin_bit_cast(vpf_u16x2, v.w & 0x7fff7fffu);
    const vpf_u16x2 m = __builtin_elementwise_max(__builtin_elementwise_max(a, b), __builtin_elementwise_max(c, d));
    return max((uint32_t)m.x, (uint32_t)m.y);
}

// 8 packed bf16 values -> 8 e4m3 bytes of RNE(x * 2^-E) (E = the block exponent), by gfx950's
// v_cvt_scalef32_pk_fp8_bf16: the packed bf16 pair converted with the block scale in one instruction (4 per 8 values
// instead of 8 unpacks + 8 multiplies + 4 v_cvt_pk_fp8_f32). The instruction divides by its scale operand: with scale
// 2^E it is bit-identical to RNE(x * 2^-E) for every E in [-127, 125], E = -127 included (see sc below) (tools/micro/cvt_scalef.py on the MI355X: 0 of
// 1,048,576 pairs differ; with 2^-E 98.9 % of them differ: profiles/r4_lab/cvt_scalef_probe.txt).
typedef __bf16 vpf_bf16x2 __attribute__((ext_vector_type(2)));
typedef short vpf_s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint2 mx8_pack8(uint4 v, int E) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    // 2^E as an fp32 bit pattern: a normal float for E in [-126, 125]. E = -127 (a block whose max is below 2^-118,
    // e.g. all zeros) gives the bit pattern of +0.0, not 2^-127: the result is still RNE(x * 2^127) because the
    // instruction takes only the exponent field of its scale operand (tools/micro/cvt_scalef.py covers E = -127 among
    // its random blocks: 0 differences), which this code relies on.
    const float sc = __uint_as_float((uint32_t)(127 + E) << 23);
    vpf_s16x2 lo = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(vpf_s16x2{0, 0}, __builtin_bit_cast(vpf_bf16x2, w[0]), sc,
                                                             false);
    lo = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(lo, __builtin_bit_cast(vpf_bf16x2, w[1]), sc, true);
    vpf_s16x2 hi = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(vpf_s16x2{0, 0}, __builtin_bit_cast(vpf_bf16x2, w[2]), sc,
                                                             false);
    hi = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(hi, __builtin_bit_cast(vpf_bf16x2, w[3]), sc, true);
    return make_uint2(__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi));
}

// 8 consecutive bf16 values of one row (one lane) -> 8 e4m3 bytes; the 32-value block is the lane's DPP quad
// (lanes 4q .. 4q+3 hold columns 32b .. 32b+31 in order). Every lane of the quad must execute this.
__device__ __forceinline__ uint2 mx8_quant8(uint4 v, uint32_t& e8m0) {
    uint32_t am = mx8_amax8(v);
    am = max(am, (uint32_t)__builtin_amdgcn_mov_dpp((int)am, 0xB1, 0xF, 0xF, false));   // quad_perm(1,0,3,2)
    am = max(am, (uint32_t)__builtin_amdgcn_mov_dpp((int)am, 0x4E, 0xF, 0xF, false));   // quad_perm(2,3,0,1)
    const int E = mx8_block_exp(am);
    e8m0 = (uint32_t)(E + 127);
    return mx8_pack8(v, E);
}

}  // namespace vpf
