// Micro-benchmark (design aid): issue rate of packed-f32 VALU (v_pk_fma_f32 / v_pk_mul_f32) against scalar
// v_fma_f32 doing the same FLOPs, wave64, 1 / 2 / 4 waves per SIMD. Each thread runs ITER iterations of 8
// independent chains; time = one launch (HIP events, median of 9).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITER = 4096;
__global__ void k_pk(float* out, float a, float b) {
    f2 x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = f2{(float)threadIdx.x + k, (float)k};
    const f2 va = {a, a}, vb = {b, b};
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = __builtin_elementwise_fma(x[k], va, vb);
    }
    f2 s = x[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) s += x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y;
}
__global__ void k_sc(float* out, float a, float b) {
    float x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = (float)threadIdx.x + k;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            float y = x[k];
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(y) : "v"(a), "v"(b));
            x[k] = y;
        }
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_pkasm(float* out, float a, float b) {
    f2 x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = f2{(float)threadIdx.x + k, (float)k};
    const f2 va = {a, a}, vb = {b, b};
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x[k]) : "v"(va), "v"(vb));
    }
    f2 s = x[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) s += x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y;
}
int main() {
    float* out; hipMalloc(&out, 256 * 1024 * 4 * 16);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    int cus = 256;
    for (int wps : {1, 2, 4}) {            // waves per SIMD: blocks of 256 threads (4 waves = one per SIMD)
        const int blocks = cus * wps;
        for (int v = 0; v < 3; ++v) {
            std::vector<float> t;
            for (int r = 0; r < 9; ++r) {
                hipEventRecord(e0);
                if (v == 0) hipLaunchKernelGGL(k_pk, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 0.001f);
                else if (v == 1) hipLaunchKernelGGL(k_pkasm, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 0.001f);
                else hipLaunchKernelGGL(k_sc, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 0.001f);
                hipEventRecord(e1); hipEventSynchronize(e1);
                float ms; hipEventElapsedTime(&ms, e0, e1); t.push_back(ms);
            }
            std::sort(t.begin(), t.end());
            const double flops = 2.0 * 16 * ITER * 256.0 * blocks;   // 16 fp32 FMA lanes per thread per iteration
            printf("%-22s waves/SIMD %d  median %.3f ms  %.1f TFLOP/s fp32\n",
                   v == 0 ? "v_pk_fma_f32 (builtin)" : v == 1 ? "v_pk_fma_f32 (asm)" : "v_fma_f32 x2 (asm)", wps, t[4],
                   flops / (t[4] * 1e-3) / 1e12);
        }
    }
    return 0;
}
