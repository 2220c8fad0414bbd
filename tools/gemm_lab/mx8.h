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

// |x| max of 8 packed bf16 values, as |bf16| bits (integer order = magnitude order)
__device__ __forceinline__ uint32_t mx8_amax8(uint4 v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t am = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) am = max(am, max(w[e] & 0x7fffu, (w[e] >> 16) & 0x7fffu));
    return am;
}

// 8 packed bf16 values -> 8 e4m3 bytes of x * 2^-E (E = the block exponent)
__device__ __forceinline__ uint2 mx8_pack8(uint4 v, int E) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    const float inv = __uint_as_float((uint32_t)(127 - E) << 23);     // 2^-E (normal for E in [-127, 125])
    int lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f((bf16_t)(w[0] & 0xffff)) * inv, bf2f((bf16_t)(w[0] >> 16)) * inv, 0,
                                             false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f((bf16_t)(w[1] & 0xffff)) * inv, bf2f((bf16_t)(w[1] >> 16)) * inv, lo,
                                         true);
    int hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f((bf16_t)(w[2] & 0xffff)) * inv, bf2f((bf16_t)(w[2] >> 16)) * inv, 0,
                                             false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f((bf16_t)(w[3] & 0xffff)) * inv, bf2f((bf16_t)(w[3] >> 16)) * inv, hi,
                                         true);
    return make_uint2((uint32_t)lo, (uint32_t)hi);
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
