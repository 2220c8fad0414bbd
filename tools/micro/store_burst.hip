// Micro-benchmark (design aid): cycles a 512-thread workgroup needs to issue and complete a GEMM-epilogue store
// burst (128 KiB = 16 x 1 KiB dwordx4 stores per wave, 8 rows x 128 B per instruction), stamped in-kernel with
// s_memtime around the burst + s_waitcnt vmcnt(0), for 1 / 32 / 256 / 512 concurrent workgroups (one per CU up
// to 256). Also the same burst with global_store_dwordx4 ... nt and buffer stores. Median over workgroups.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
template <int KIND>
__global__ __launch_bounds__(512) void k_burst(char* out, unsigned long long* t, int ld) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    char* base = out + (size_t)blockIdx.x * 256 * ld + (size_t)(wid >> 2) * 128 * ld + (wid & 3) * 128;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 v = {(unsigned)lane, (unsigned)wid, blockIdx.x, 7u};
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        char* p = base + (size_t)(it * 8 + (lane >> 3)) * ld + (lane & 7) * 16;
        if constexpr (KIND == 0) *reinterpret_cast<u32x4*>(p) = v;
        else if constexpr (KIND == 1) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
        v.x += 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    const unsigned long long t2 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { t[blockIdx.x * 2] = t1 - t0; t[blockIdx.x * 2 + 1] = t2 - t0; }
}
int main() {
    const int ld = 3072 * 2;   // FC1 output row pitch (bytes)
    char* out; (void)hipMalloc(&out, (size_t)1024 * 256 * ld);
    unsigned long long* t; (void)hipMalloc(&t, 1024 * 2 * 8);
    std::vector<unsigned long long> h(2048);
    for (int kind = 0; kind < 2; ++kind)
        for (int nwg : {1, 8, 32, 128, 256}) {
            std::vector<double> wv, bv;
            for (int r = 0; r < 5; ++r) {
                if (kind == 0) hipLaunchKernelGGL(k_burst<0>, dim3(nwg), dim3(512), 0, 0, out, t, ld);
                else hipLaunchKernelGGL(k_burst<1>, dim3(nwg), dim3(512), 0, 0, out, t, ld);
                (void)hipDeviceSynchronize();
                (void)hipMemcpy(h.data(), t, nwg * 16, hipMemcpyDeviceToHost);
                if (r == 0) continue;   // warm-up
                for (int b = 0; b < nwg; ++b) { wv.push_back((double)h[2 * b]); bv.push_back((double)h[2 * b + 1]); }
            }
            std::sort(wv.begin(), wv.end()); std::sort(bv.begin(), bv.end());
            printf("%-6s nwg=%4d  wave0 issue+complete: median %.0f cyc (max %.0f); whole workgroup: median %.0f cyc -> %.1f B/cyc/CU\n",
                   kind ? "nt" : "plain", nwg, wv[wv.size() / 2], wv.back(), bv[bv.size() / 2], 131072.0 / bv[bv.size() / 2]);
        }
    return 0;
}
