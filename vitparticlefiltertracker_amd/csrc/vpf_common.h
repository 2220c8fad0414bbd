// Shared device helpers for libvpf (gfx950 / CDNA4 only).
//
// * bf16 <-> f32 conversion (round-to-nearest-even; hipcc lowers the __bf16 cast to v_cvt_pk_bf16_f32).
// * Philox4x32-10 and the fixed fp32 elementary functions of SPEC.md S1/S2. These must produce the
//   same bits as oracle/pf_oracle.c: every fused multiply-add is an explicit fmaf and the translation
//   units that use them compile with `#pragma clang fp contract(off)`.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define VPF_API extern "C" __attribute__((visibility("default")))

// Launch helper: return the launch status as the C-ABI result (0 = hipSuccess).
#define VPF_RETURN_LAUNCH() return (int)hipGetLastError()

namespace vpf {

typedef unsigned short bf16_t;  // storage type of bf16 in global memory

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
    __bf16 b = (__bf16)f;
    return __builtin_bit_cast(bf16_t, b);
}
// two floats -> packed bf16x2 (lo in bits 0..15), round-to-nearest-even: ONE v_cvt_pk_bf16_f32 (two scalar
// casts + shift/or cost four VALU instructions).
typedef __bf16 vpf_bf16x2 __attribute__((ext_vector_type(2)));
typedef float vpf_f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(vpf_f32x2{lo, hi}, vpf_bf16x2));
}

// ---------------- Philox4x32-10 (SPEC S1) ----------------
struct u32x4 { uint32_t v[4]; };

__device__ __forceinline__ u32x4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                               uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    u32x4 o; o.v[0] = c0; o.v[1] = c1; o.v[2] = c2; o.v[3] = c3;
    return o;
}

__device__ __forceinline__ float uniform01(uint32_t r) {
    return (float)(2u * (r >> 9) + 1u) * 5.9604644775390625e-8f;
}

// ln(x), x in (0, 1]; Cephes-style polynomial, explicit fmaf (SPEC S2)
__device__ __forceinline__ float fixed_logf(float x) {
    const uint32_t b = __float_as_uint(x);
    int e = (int)((b >> 23) & 0xff) - 126;
    float m = __uint_as_float((b & 0x007fffffu) | 0x3f000000u);
    if (m < 0.70710678118654752f) { e -= 1; m = m + m - 1.0f; } else { m = m - 1.0f; }
    const float z = m * m;
    float p = 7.0376836292e-2f;
    p = fmaf(p, m, -1.1514610310e-1f);
    p = fmaf(p, m, 1.1676998740e-1f);
    p = fmaf(p, m, -1.2420140846e-1f);
    p = fmaf(p, m, 1.4249322787e-1f);
    p = fmaf(p, m, -1.6668057665e-1f);
    p = fmaf(p, m, 2.0000714765e-1f);
    p = fmaf(p, m, -2.4999993993e-1f);
    p = fmaf(p, m, 3.3333331174e-1f);
    float y = (m * z) * p;
    const float fe = (float)e;
    y = fmaf(fe, -2.12194440e-4f, y);
    y = fmaf(z, -0.5f, y);
    float r = m + y;
    return fmaf(fe, 0.693359375f, r);
}

// exp(x): Cephes-style, explicit fmaf; exact 0 below -87 (SPEC S2, S5)
__device__ __forceinline__ float fixed_expf(float x) {
    if (x < -87.0f) return 0.0f;
    if (x > 88.0f) x = 88.0f;
    const float fn = floorf(fmaf(x, 1.44269504088896341f, 0.5f));
    float r = fmaf(fn, -0.693359375f, x);
    r = fmaf(fn, 2.12194440e-4f, r);
    const float z = r * r;
    float p = 1.9875691500e-4f;
    p = fmaf(p, r, 1.3981999507e-3f);
    p = fmaf(p, r, 8.3334519073e-3f);
    p = fmaf(p, r, 4.1665795894e-2f);
    p = fmaf(p, r, 1.6666665459e-1f);
    p = fmaf(p, r, 5.0000001201e-1f);
    float y = fmaf(p, z, r) + 1.0f;
    const int n = (int)fn;
    const int n1 = n / 2, n2 = n - n1;
    y = y * __uint_as_float((uint32_t)(n1 + 127) << 23);
    y = y * __uint_as_float((uint32_t)(n2 + 127) << 23);
    return y;
}

// (cos, sin)(2*pi*u), u in [0, 1) (SPEC S2)
__device__ __forceinline__ void fixed_sincos2pi(float u, float& c_out, float& s_out) {
    const float t = u * 4.0f;
    const float q = floorf(t);
    const float r = t - q;
    const float a = (r - 0.5f) * 1.57079632679489662f;
    const float z = a * a;
    float sp = -1.9515295891e-4f;
    sp = fmaf(sp, z, 8.3321608736e-3f);
    sp = fmaf(sp, z, -1.6666654611e-1f);
    const float sa = fmaf(a * z, sp, a);
    float cp = 2.443315711809948e-5f;
    cp = fmaf(cp, z, -1.388731625493765e-3f);
    cp = fmaf(cp, z, 4.166664568298827e-2f);
    const float ca = fmaf(z * z, cp, fmaf(z, -0.5f, 1.0f));
    const float h = 0.70710678118654752f;
    const float c0 = (ca - sa) * h, s0 = (ca + sa) * h;
    const int qi = (int)q & 3;
    float c, s;
    if (qi == 0) { c = c0; s = s0; }
    else if (qi == 1) { c = -s0; s = c0; }
    else if (qi == 2) { c = -c0; s = -s0; }
    else { c = s0; s = -c0; }
    c_out = c; s_out = s;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

}  // namespace vpf
