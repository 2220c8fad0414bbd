"""Both bf16 GEMM K loops without the past-the-end operand re-stages: the last two K-steps are peeled (compile-time
modes) so that K-tile nk - 1 is not DMA'd again into its own slots (kernel 1: 3 x 32 KiB per tile; kernel 5: 6 half
tiles = 96 KiB per tile, 12.5 % of a K = 768 tile's operand bytes), with the counted vmcnt of those phases lowered to
what is then in flight. The loop then ends with nothing outstanding (the product's closing vmcnt(0) waits for the
re-stages issued in the last K-step). Bit-identical by construction (the re-stages wrote identical bytes)."""
K1_OLD = open(__file__.replace('nodup.py', 'nodup_k1_old.txt')).read()
K5_OLD = open(__file__.replace('nodup.py', 'nodup_k5_old.txt')).read()

K1_NEW = r'''    // MODE 0: refill B(t+1), A(t+2); MODE 1 (t = nk - 2): B(t+1) only; MODE 2 (t = nk - 1): nothing (round 6: no
    // past-the-end re-stage of K-tile nk - 1, so nothing is in flight when the loop ends)
    auto kstep = [&](int kt, auto mode_c) {
        constexpr int MODE = decltype(mode_c)::value;
        // issue order: A0 B0 A1 | per K-tile t: B(t+1) A(t+2). A(kt), B(kt) are older than everything but A(kt+1)
        // (4 pieces per wave) until the last two K-tiles, where the tail is B / aux only.
        if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (nk >= 2 && kt == nk - 2) load_aux();
        if (wide && kt == nk - 1) load_planes(planes_lds);   // slot of A(nk-2): free after this barrier
        const char* la = smem + (kt % 3) * OPERAND_BYTES;
        const char* lb = smem + (3 + (kt & 1)) * OPERAND_BYTES;
        bf16x8 a[2][8], b[2][4];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int row = wn * 64 + j * 16 + fr;
                const int ch = (ks * 4 + fq) ^ ((row >> 1) & 7);
                b[ks][j] = *reinterpret_cast<const bf16x8*>(lb + row * 128 + ch * 16);
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int row = wm * 128 + i * 16 + fr;
                const int ch = (ks * 4 + fq) ^ ((row >> 1) & 7);
                a[ks][i] = *reinterpret_cast<const bf16x8*>(la + row * 128 + ch * 16);
            }
        }
        if constexpr (MODE <= 1) stage_b(kt + 1);
        if constexpr (MODE == 0) stage_a(kt + 2);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[ks][j], a[ks][i], acc[j][i], 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 24, 0);   // the 24 fragment reads
        if constexpr (MODE <= 1) __builtin_amdgcn_sched_group_barrier(0x020, 4, 0);    // B(t+1)'s DMA
        if constexpr (MODE == 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {                          // 16 MFMAs per A(t+2) DMA issue
                __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            }
        }
    };
    for (int kt = 0; kt < nk - 2; ++kt) kstep(kt, std::integral_constant<int, 0>{});
    if (nk >= 2) kstep(nk - 2, std::integral_constant<int, 1>{});
    kstep(nk - 1, std::integral_constant<int, 2>{});
'''

K5_NEW = r'''    // MODE 0: the steady state; MODE 1 (kt = nk - 2): q2 / q3 stage nothing (they would re-stage K-tile nk - 1), q3's
    // wait leaves 2 half-tiles in flight; MODE 2 (kt = nk - 1): nothing staged, q0 leaves 1 half-tile, q1 none (round 6)
    auto kstep = [&](int kt, auto mode_c) {
        constexpr int MODE = decltype(mode_c)::value;
        const char* buf = smem + (kt & 1) * 4 * HALF;
        i32x4 fa0[2][4], fa1[2][4], fb0[2][2], fb1[2][2];
        // q0: (mh0, nh0)
        read_a(fa0, buf);
        read_b(fb0, buf + HALF);
        if constexpr (MODE <= 1) {
            stage(2, kt + 1);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        }
        bar();
        mfma_quadrant(fa0, fb0, 0, 0);
        bar();
        // q1: (mh0, nh1)
        read_b(fb1, buf + 2 * HALF);
        if constexpr (MODE <= 1) {
            stage(3, kt + 1);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        bar();
        mfma_quadrant(fa0, fb1, 0, 1);
        bar();
        // q2: (mh1, nh1)
        read_a(fa1, buf + 3 * HALF);
        if constexpr (MODE == 0) stage(0, kt + 2);
        bar();
        mfma_quadrant(fa1, fb1, 1, 1);
        bar();
        // q3: (mh1, nh0)
        if constexpr (MODE == 0) {
            stage(1, kt + 2);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else if constexpr (MODE == 1) {
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        }
        bar();
        mfma_quadrant(fa1, fb0, 1, 0);
        bar();
    };
    for (int kt = 0; kt < nk - 2; ++kt) kstep(kt, std::integral_constant<int, 0>{});
    if (nk >= 2) kstep(nk - 2, std::integral_constant<int, 1>{});
    kstep(nk - 1, std::integral_constant<int, 2>{});
    if (wm == 0) __builtin_amdgcn_s_barrier();   // matches wm = 1's offset barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // nothing outstanding (no past-the-end re-stage)
'''
EDITS = [
    ("gemm_bf16.hip", K1_OLD, K1_NEW),
    ("gemm_bf16.hip", K5_OLD, K5_NEW),
    ("gemm_bf16.hip", "#include <algorithm>\n", "#include <algorithm>\n#include <type_traits>\n"),
]
