// Which SIMD each wave of a workgroup lands on (design aid for the key-streamed N > 256 attention): WG waves x 64
// threads, LDS sized so that K workgroups share a CU; every wave records HW_ID (wave 3:0, simd 5:4, cu 11:8, sh 12,
// se 15:13) and XCC_ID, then sleeps so that every workgroup is resident at once. Prints, per launch shape, how many
// CUs carry each per-SIMD wave count pattern.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <string>
#include <vector>
__global__ void k(unsigned* out) {
    extern __shared__ char smem[];
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        out[2 * w] = __builtin_amdgcn_s_getreg(0xF804);
        out[2 * w + 1] = __builtin_amdgcn_s_getreg(0xF814);
        smem[threadIdx.x] = 1;
    }
    __syncthreads();
    for (int i = 0; i < 200; ++i) __builtin_amdgcn_s_sleep(127);
}
static void run(int waves, int lds, int per_cu) {
    const int G = 256 * per_cu;
    unsigned* d;
    const int nw = G * waves;
    hipMalloc(&d, 2 * nw * sizeof(unsigned));
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL(k, dim3(G), dim3(64 * waves), lds, 0, d);
    std::vector<unsigned> h(2 * nw);
    hipMemcpy(h.data(), d, 2 * nw * sizeof(unsigned), hipMemcpyDeviceToHost);
    hipFree(d);
    std::map<unsigned, std::vector<int>> cu;   // (xcc, se, sh, cu) -> waves per simd
    for (int w = 0; w < nw; ++w) {
        const unsigned hw = h[2 * w], xcc = h[2 * w + 1] & 0xF;
        const unsigned key = (xcc << 16) | (((hw >> 13) & 7) << 12) | (((hw >> 12) & 1) << 8) | ((hw >> 8) & 0xF);
        auto& v = cu[key];
        if (v.empty()) v.assign(4, 0);
        v[(hw >> 4) & 3]++;
    }
    std::map<std::string, int> pat;
    for (auto& [key, v] : cu) {
        char b[64];
        snprintf(b, sizeof b, "%d,%d,%d,%d", v[0], v[1], v[2], v[3]);
        pat[b]++;
    }
    printf("%d-wave workgroups, %d B LDS (%d per CU intended): %zu CUs; waves per SIMD pattern -> CUs:", waves, lds,
           per_cu, cu.size());
    for (auto& [p, n] : pat) printf("  [%s] x%d", p.c_str(), n);
    printf("\n");
}
int main() {
    run(6, 72 * 1024, 2);
    run(4, 48 * 1024, 3);
    run(8, 57 * 1024, 2);
    run(7, 57 * 1024, 2);
    return 0;
}
