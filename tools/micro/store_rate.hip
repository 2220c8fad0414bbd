// Micro-benchmark (design aid): per-CU global store throughput for a GEMM-epilogue-sized burst.
// Each 512-thread workgroup writes `kb` KiB: every wave issues 16-B-per-lane stores (1 KiB per
// wave-instruction, 8 rows x 128 B like the GEMM epilogue) or 8-B-per-lane MFMA-layout stores (16 rows x 32 B).
// Grid = nwg workgroups (1 per CU at most); time = one launch, HIP events, median of 20.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
__global__ __launch_bounds__(512) void k_store16(uint4* out, int per_wave, int row_bytes) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    char* base = reinterpret_cast<char*>(out) + (size_t)blockIdx.x * 8 * per_wave * 1024 + (size_t)wid * per_wave * 1024;
    const uint4 v = make_uint4(lane, wid, blockIdx.x, 7);
    for (int i = 0; i < per_wave; ++i)
        *reinterpret_cast<uint4*>(base + i * 1024 + lane * 16) = v;
}
__global__ __launch_bounds__(512) void k_store8(uint2* out, int per_wave, int ld) {
    // 16 rows x 32 B per instruction: lane (fr = lane & 15, fq = lane >> 4) -> row fr, bytes fq*8..+8
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int fr = lane & 15, fq = lane >> 4;
    char* base = reinterpret_cast<char*>(out) + (size_t)blockIdx.x * 8 * per_wave * 512 + (size_t)wid * per_wave * 512;
    const uint2 v = make_uint2(lane, wid);
    for (int i = 0; i < per_wave; ++i) {
        // instruction i covers rows (i/4)*16 + fr of a 128-B-wide strip, column chunk (i%4)*32 + fq*8
        char* p = base + ((size_t)((i >> 2) * 16 + fr) * 128) + (i & 3) * 32 + fq * 8;
        *reinterpret_cast<uint2*>(p) = v;
    }
}
int main() {
    const size_t bytes = (size_t)1 << 31;
    void* buf; hipMalloc(&buf, bytes); hipMemset(buf, 0, bytes);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int kind = 0; kind < 2; ++kind)
        for (int nwg : {1, 64, 256}) {
            for (int kbw : {1, 4, 16, 64}) {   // KiB per wave: 16 -> 128 KiB per workgroup (one 256x256 bf16 tile)
                const int per_wave = kind == 0 ? kbw : kbw * 2;
                std::vector<float> t;
                for (int r = 0; r < 20; ++r) {
                    hipEventRecord(e0);
                    if (kind == 0) hipLaunchKernelGGL(k_store16, dim3(nwg), dim3(512), 0, 0, (uint4*)buf, per_wave, 0);
                    else hipLaunchKernelGGL(k_store8, dim3(nwg), dim3(512), 0, 0, (uint2*)buf, per_wave, 0);
                    hipEventRecord(e1); hipEventSynchronize(e1);
                    float ms; hipEventElapsedTime(&ms, e0, e1); t.push_back(ms);
                }
                std::sort(t.begin(), t.end());
                const double tot = (double)nwg * 8 * kbw * 1024;
                printf("%s nwg=%5d  %3d KiB/WG  median %.2f us  -> %.1f GB/s total, %.1f GB/s per WG-wave-of-CUs\n",
                       kind == 0 ? "dwordx4 8x128B" : "dwordx2 16x32B", nwg, 8 * kbw, t[10] * 1e3, tot / (t[10] * 1e-3) / 1e9,
                       tot / (t[10] * 1e-3) / 1e9 / std::min(nwg, 256));
            }
        }
    return 0;
}
