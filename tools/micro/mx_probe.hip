// Operand-layout probe for v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3): one wave per configuration runs a
// single MFMA on caller-supplied per-lane registers (A, B: 8 dwords = 32 bytes per lane; scale VGPRs) and
// stores the 4 accumulator registers per lane. tools/micro/mx_probe.py designs the inputs and reads the maps.
// Build: hipcc --offload-arch=gfx950 -O2 -shared -fPIC tools/micro/mx_probe.hip -o tools/micro/libmxprobe.so
#include <hip/hip_runtime.h>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int OA, int OB>
__global__ void k_probe(const i32x8* A, const i32x8* B, const int* SA, const int* SB, f32x4* D) {
    const int c = blockIdx.x, l = threadIdx.x;
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    D[c * 64 + l] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A[c * 64 + l], B[c * 64 + l], z, 0, 0, OA,
                                                                      SA[c * 64 + l], OB, SB[c * 64 + l]);
}

extern "C" int mx_probe(const void* A, const void* B, const int* SA, const int* SB, void* D, int cfgs, int opsel_a,
                        int opsel_b, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    const i32x8* a = (const i32x8*)A;
    const i32x8* b = (const i32x8*)B;
    f32x4* d = (f32x4*)D;
#define P(OA, OB) if (opsel_a == OA && opsel_b == OB) hipLaunchKernelGGL((k_probe<OA, OB>), dim3(cfgs), dim3(64), 0, s, a, b, SA, SB, d)
    P(0, 0); P(1, 0); P(2, 0); P(3, 0); P(0, 1); P(0, 2); P(0, 3);
#undef P
    return (int)hipGetLastError();
}
