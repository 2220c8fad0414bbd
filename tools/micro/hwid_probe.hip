// Which workgroups share a CU, and what HW_ID says about them (design aid for a persistent attention whose two
// resident workgroups per CU run half a unit apart). 512 workgroups of 512 threads with 57 KiB of LDS each (two per
// CU, like the attention kernel); each records HW_ID (cu 11:8, sh 12, se 15:13, tg 19:16) and XCC_ID.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>
__global__ __launch_bounds__(512) void k(unsigned* out) {
    extern __shared__ char smem[];
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = __builtin_amdgcn_s_getreg(0xF804);
        out[2 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg(0xF814);
        smem[0] = 1;
    }
    __syncthreads();
    for (int i = 0; i < 200; ++i) __builtin_amdgcn_s_sleep(127);   // stay resident: every workgroup runs at once
}
int main() {
    const int G = 512;
    unsigned* d;
    hipMalloc(&d, 2 * G * sizeof(unsigned));
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL(k, dim3(G), dim3(512), 57344, 0, d);
    std::vector<unsigned> h(2 * G);
    hipMemcpy(h.data(), d, 2 * G * sizeof(unsigned), hipMemcpyDeviceToHost);
    std::map<unsigned, std::vector<int>> per_cu;
    for (int b = 0; b < G; ++b) {
        const unsigned hw = h[2 * b], xcc = h[2 * b + 1] & 0xF;
        per_cu[(xcc << 8) | ((hw >> 8) & 0xFF)].push_back(b);
    }
    int two = 0, other = 0, tg_diff = 0, half = 0;
    for (auto& [key, bs] : per_cu) {
        if (bs.size() == 2) {
            ++two;
            const unsigned t0 = (h[2 * bs[0]] >> 16) & 0xF, t1 = (h[2 * bs[1]] >> 16) & 0xF;
            tg_diff += (t0 & 1) != (t1 & 1);
            half += (bs[0] < 256) != (bs[1] < 256);
        } else {
            ++other;
        }
    }
    printf("CUs seen %zu: with 2 workgroups %d, other %d; pairs whose TG_ID parity differs %d; pairs split by block < 256: %d\n",
           per_cu.size(), two, other, tg_diff, half);
    int shown = 0;
    for (auto& [key, bs] : per_cu) {
        if (shown++ >= 6) break;
        printf("cu key %04x:", key);
        for (int b : bs) printf("  block %d tg %u", b, (h[2 * b] >> 16) & 0xF);
        printf("\n");
    }
    return 0;
}
