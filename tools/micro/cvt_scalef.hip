// Probe (design aid): does v_cvt_scalef32_pk_fp8_bf16 (gfx950) reproduce the MX quantiser's element rule
// RNE(x * 2^-E) of mx8.h's mx8_pack8 on packed bf16 inputs, and with which scale operand (2^E or 2^-E)?
// Built by tools/micro/cvt_scalef.py (hipcc -shared), run on the GPU box.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef short s2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float bf2f(uint32_t h) { return __uint_as_float(h << 16); }

// out[i] = 4 bytes: reference (mx8_pack8's rule) of the two bf16 values of in[i] in bytes 0-1, the scaled
// conversion with scale = 2^E in bytes 2-3 (variant 0) or 2^-E (variant 1)
__global__ void k_probe(const uint32_t* in, const int* E, uint32_t* out, int n, int variant) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t w = in[i];
    const int e = E[i];
    const float inv = __uint_as_float((uint32_t)(127 - e) << 23);
    const int ref = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(w & 0xffff) * inv, bf2f(w >> 16) * inv, 0, false) & 0xffff;
    const float sc = variant == 0 ? __uint_as_float((uint32_t)(127 + e) << 23) : inv;
    const s2_t r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(s2_t{0, 0}, __builtin_bit_cast(bf16x2_t, w), sc, false);
    const uint32_t got = __builtin_bit_cast(uint32_t, r) & 0xffff;
    out[i] = (uint32_t)ref | (got << 16);
}

extern "C" int probe(const uint32_t* in, const int* E, uint32_t* out, int n, int variant) {
    hipLaunchKernelGGL(k_probe, dim3((n + 255) / 256), dim3(256), 0, 0, in, E, out, n, variant);
    return (int)hipDeviceSynchronize();
}
