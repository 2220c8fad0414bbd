"""(GEMM-only form: the attention keeps its unit order and only advances the counter) Alternating traversal order between consecutive bf16 GEMM / attention launches, so each kernel starts on the rows
the previous one wrote last (still in that XCD's L2 or in the Infinity Cache). Every launch of vpf_gemm_bf16 and of the
N <= 256 attention takes the next parity of a host counter (the launch sequence is fixed when the frame's graph is
captured): odd launches walk each XCD's contiguous tile range (GEMM) / unit slice (attention) backwards. The attention
also gets the GEMMs' XCD slicing (blocks of XCD x take units of the contiguous slice x instead of every 8th unit).
Outputs do not depend on the order (bit-identical)."""
EDITS = [
    ("gemm_common.h", '''__device__ __forceinline__ void tile_of(int M, int N, int group, int& m0, int& n0) {
    const int nwg = gridDim.x, bid = blockIdx.x;
    tile_of_lid(M, N, group, xcd_first(nwg, bid & 7) + (bid >> 3), m0, n0);
}''', '''__device__ __forceinline__ void tile_of(int M, int N, int group, int& m0, int& n0) {
    const int nwg = gridDim.x, bid = blockIdx.x;
    const bool rev = group < 0;
    const int g = rev ? ~group : group;
    const int x = bid & 7, len = (nwg >> 3) + (x < (nwg & 7) ? 1 : 0), j = bid >> 3;
    tile_of_lid(M, N, g, xcd_first(nwg, x) + (rev ? len - 1 - j : j), m0, n0);
}'''),
    ("gemm_bf16.hip", '''static int g_group = -1;   // -1: per-shape default''', '''static int g_group = -1;   // -1: per-shape default
static unsigned g_launch_seq = 0;
int vpf_next_dir() { return (int)(g_launch_seq++ & 1u); }'''),
    ("gemm_bf16.hip", '''    const int group = tile_group_for(N, epilogue);
    const int m = (int)M, n = (int)N, k = (int)K;''', '''    const int group = vpf_next_dir() ? ~tile_group_for(N, epilogue) : tile_group_for(N, epilogue);
    const int m = (int)M, n = (int)N, k = (int)K;'''),
    ("attention.hip", '''    uint8_t* __restrict__ out8 = nullptr, int ld8 = 0, uint8_t* __restrict__ s8 = nullptr, int lds8 = 0) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int NP = (N + 31) & ~31;
    const int NT = NP >> 5;              // 32-key chunks
    char* Ks = smem;
    char* Vs = smem + NP * ROWB;
    const int bh = blockIdx.x;''', '''    uint8_t* __restrict__ out8 = nullptr, int ld8 = 0, uint8_t* __restrict__ s8 = nullptr, int lds8 = 0, int dir = 0) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int NP = (N + 31) & ~31;
    const int NT = NP >> 5;              // 32-key chunks
    char* Ks = smem;
    char* Vs = smem + NP * ROWB;
    int bh;
    {
        const int nwg = gridDim.x, bid = blockIdx.x;
        const int x = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
        const int len = q8 + (x < r8 ? 1 : 0), j = bid >> 3;
        const int first = x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8;
        (void)first; (void)len; (void)j; (void)dir;
        bh = bid;
    }'''),
    ("attention.hip", '''                           (uint8_t*)nullptr, 0, (uint8_t*)nullptr, 0);''',
     '''                           (uint8_t*)nullptr, 0, (uint8_t*)nullptr, 0, vpf_next_dir());'''),
    ("attention.hip", '''namespace {

typedef const __attribute__((address_space(1))) void* gptr_t;''', '''int vpf_next_dir();   // gemm_bf16.hip: the shared launch-parity counter

namespace {

typedef const __attribute__((address_space(1))) void* gptr_t;'''),
]
