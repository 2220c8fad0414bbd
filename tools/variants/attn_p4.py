"""N <= 256 bf16 attention with three units in flight per CU (k_attn_pipe4, round 6): one 4-wave workgroup per
(particle, head), each wave two query strips in turn (strips w and w + 4), the head's K / V image in LDS cut at the
16-row tail tile when N % 32 is 1..16 (N = 197: 208 rows, 52 KiB: three workgroups per CU, three waves per SIMD).
The first strip runs the product's chunk loop (counted waits + barriers as the chunks land), the second one over the
landed image without barriers. Layout [V image][K image]: the steps' reads past the tail tile (V rows 16..31 of the
last chunk land in the K image: finite, times probability 0; K rows past the image: out of the workgroup's LDS range,
scores masked to -inf) need no padding. The MX8-output path keeps k_attn_bf16_pipe. The N sweep
(r6_lab/attn_nsweep.txt) says a unit's fixed cost dominates at two resident units per CU; this puts three in flight
with the 32-query steps (round 6's 16-query-strip form of three units, attn_q16, lost on the 16x16x32 steps)."""
_K = r'''
// ---- lab: k_attn_pipe4 (tools/variants/attn_p4.py) ----
template <int CPB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void k_attn_pipe4(
    const bf16_t* __restrict__ qkv, bf16_t* __restrict__ out, int N, int H, float scale_log2, int q_rows, int NR) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int NP = (N + 31) & ~31;
    const int NT = NP >> 5;
    char* Vs = smem;
    char* Ks = smem + NR * ROWB;
    const int bh = blockIdx.x;
    const int b = bh / H, h = bh - (bh / H) * H;
    const int D = H * HD;
    const int64_t row0 = (int64_t)b * N;
    const bf16_t* qbase = qkv + row0 * 3 * D + h * HD;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l32 = lane & 31, hh = lane >> 5;
    const int nstrips = (q_rows + 31) >> 5;
    const int nlast = (N - 1) >> 5;
    const int sA = wid, sB = wid + 4;
    const bool w16A = sA == nlast && sA < nstrips && N - 32 * nlast <= 16;
    const bool w16B = sB == nlast && sB < nstrips && N - 32 * nlast <= 16;
    bf16x8 qa[4], qb[4];
    {
        const bf16_t* pa = w16A ? qbase + (int64_t)min(sA * 32 + (lane & 15), N - 1) * 3 * D + 8 * (lane >> 4)
                                : qbase + (int64_t)min(sA * 32 + l32, N - 1) * 3 * D + hh * 8;
        const bf16_t* pb = w16B ? qbase + (int64_t)min(sB * 32 + (lane & 15), N - 1) * 3 * D + 8 * (lane >> 4)
                                : qbase + (int64_t)min(sB * 32 + l32, N - 1) * 3 * D + hh * 8;
        const int stA = w16A ? 32 : 16, stB = w16B ? 32 : 16;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
            asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qa[ks]) : "v"(pa + (w16A ? (ks & 1) : ks) * stA));
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
            asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qb[ks]) : "v"(pb + (w16B ? (ks & 1) : ks) * stB));
    }
    {
        const int sub = lane >> 3, slot = lane & 7;
        for (int c = 0; c < NT; ++c) {
            int g = c * 4 + wid;                       // 8-row piece index inside the image
            if (8 * g >= NR) g -= 2;                   // past the tail tile: re-stage the tile's own rows (same bytes)
            const int r = 8 * g + sub;
            const bf16_t* src = qbase + (int64_t)min(r, N - 1) * 3 * D;
            __builtin_amdgcn_global_load_lds((gptr_t)(src + D + (slot ^ ((r >> 1) & 7)) * 8), (lptr_t)(Ks + g * 1024),
                                             16, 0, 0);
            __builtin_amdgcn_global_load_lds((gptr_t)(src + 2 * D + (slot ^ (((r >> 1) & 1) << 2)) * 8),
                                             (lptr_t)(Vs + g * 1024), 16, 0, 0);
        }
    }
    wait_vmcnt(2 * NT);
    asm volatile("" : "+v"(qa[0]), "+v"(qa[1]), "+v"(qa[2]), "+v"(qa[3]), "+v"(qb[0]), "+v"(qb[1]), "+v"(qb[2]),
                 "+v"(qb[3]) :: "memory");
    const int nfull = N >> 5;
    auto run_strip = [&](auto k16, auto bar_c, bf16x8 (&qf)[4], int sid, bool active) {
        constexpr bool W16 = decltype(k16)::value;
        constexpr bool BAR = decltype(bar_c)::value;
        f32x16 o0 = {}, o1 = {};
        f32x4 o16[4] = {};
        float m = -INFINITY, l = 0.f;
        auto pin_q = [&]() {
            if constexpr (W16) asm volatile("" : "+v"(qf[0]), "+v"(qf[1]) :: "memory");
            else asm volatile("" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]) :: "memory");
        };
        int c = 0;
        for (; c < nfull; ++c) {
            if constexpr (BAR) {
                if (c % CPB == 0) {
                    wait_vmcnt(2 * max(NT - c - CPB, 0));
                    __builtin_amdgcn_s_barrier();
                    pin_q();
                }
            }
            if (active) {
                if constexpr (W16) attn_step16<false>(Ks + c * 4096, Vs + c * 4096, c * 32, N, lane, qf, scale_log2, m, l, o16);
                else attn_step_pl<false>(Ks + c * 4096, Vs + c * 4096, c * 32, N, lane, qf, scale_log2, m, l, o0, o1);
            }
        }
        if (c < NT) {
            if constexpr (BAR) {
                if (c % CPB == 0) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __builtin_amdgcn_s_barrier();
                    pin_q();
                }
            }
            if (active) {
                if constexpr (W16) attn_step16<true>(Ks + c * 4096, Vs + c * 4096, c * 32, N, lane, qf, scale_log2, m, l, o16);
                else if (N - c * 32 <= 8)
                    attn_step_tail8_pl(Ks + c * 4096, Vs + c * 4096, c * 32, N, lane, qf, scale_log2, m, l, o0, o1);
                else attn_step_pl<true>(Ks + c * 4096, Vs + c * 4096, c * 32, N, lane, qf, scale_log2, m, l, o0, o1);
            }
        }
        if (!active) return;
        if constexpr (W16) {
            const float inv = 1.0f / xor32_sum(xor16_sum(l));
            const int qq = sid * 32 + (lane & 15);
            if (qq < q_rows) {
                bf16_t* orow = out + (row0 + qq) * D + h * HD + 4 * (lane >> 4);
#pragma unroll
                for (int dt = 0; dt < 4; ++dt)
                    *reinterpret_cast<uint2*>(orow + 16 * dt) = make_uint2(pack_bf2(o16[dt][0] * inv, o16[dt][1] * inv),
                                                                          pack_bf2(o16[dt][2] * inv, o16[dt][3] * inv));
            }
        } else {
            const float inv = 1.0f / xor32_sum(l);
            uint32_t gx[8], gy[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const f32x16& o = k < 4 ? o0 : o1;
                const int b4 = 4 * (k & 3);
                gx[k] = pack_bf2(o[b4] * inv, o[b4 + 1] * inv);
                gy[k] = pack_bf2(o[b4 + 2] * inv, o[b4 + 3] * inv);
            }
            uint4 ov[4];
#pragma unroll
            for (int k = 0; k < 8; k += 2) {
                const auto rx = __builtin_amdgcn_permlane32_swap(gx[k], gx[k + 1], false, false);
                const auto ry = __builtin_amdgcn_permlane32_swap(gy[k], gy[k + 1], false, false);
                ov[k >> 1] = make_uint4(rx[0], ry[0], rx[1], ry[1]);
            }
            const int q = sid * 32 + l32;
            if (q < q_rows) {
                bf16_t* orow = out + (row0 + q) * D + h * HD + 8 * hh;
#pragma unroll
                for (int k = 0; k < 4; ++k) *reinterpret_cast<uint4*>(orow + 16 * k) = ov[k];
            }
        }
    };
    if (w16A) run_strip(std::true_type{}, std::true_type{}, qa, sA, true);
    else run_strip(std::false_type{}, std::true_type{}, qa, sA, sA < nstrips);
    if (sB < nstrips) {
        asm volatile("" : "+v"(qb[0]), "+v"(qb[1]), "+v"(qb[2]), "+v"(qb[3]) :: "memory");
        if (w16B) run_strip(std::true_type{}, std::false_type{}, qb, sB, true);
        else run_strip(std::false_type{}, std::false_type{}, qb, sB, true);
    }
}

'''
_f = "attention.hip"
EDITS = [
    (_f, "// ---------------- N > 256 (ViT-L/14 @ 336: N = 577): K / V streamed through a ring, queries in blocks",
     _K + "// ---------------- N > 256 (ViT-L/14 @ 336: N = 577): K / V streamed through a ring, queries in blocks"),
    (_f, """    if (N <= 256) {
        static bool pipe_attr = false;   // benign race: idempotent attribute set""",
     """    if (N <= 256) {
        const int t32 = N & 31;
        const int NR = (t32 >= 1 && t32 <= 16) ? NP - 16 : NP;
        static bool p4_attr = false;
        if (!p4_attr) {
            (void)hipFuncSetAttribute((const void*)k_attn_pipe4<PIPE_CPB>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      160 * 1024);
            p4_attr = true;
        }
        hipLaunchKernelGGL((k_attn_pipe4<PIPE_CPB>), dim3((unsigned)(B * H)), dim3(256), (size_t)NR * ROWB * 2,
                           (hipStream_t)stream, qkv, reinterpret_cast<bf16_t*>(out), N, H, scale_log2, q_rows, NR);
        VPF_RETURN_LAUNCH();
    }
    if (N <= 256) {
        static bool pipe_attr = false;   // benign race: idempotent attribute set"""),
]
