"""proj / FC2 (k_gemm_bf16, EPI_BIAS_RESIDUAL): right after the barrier of K-step nk - 3 each wave touches the 128 lines
of its residual slice (two global_load_dword, one lane per 128-B line, results discarded), so the residual loads issued
after the K loop hit L2 instead of HBM. Round 6 probe: the residual loads cost proj 0.11 ms / FC2 0.12 ms per launch
(r6_lab/gemm_residual_probes.txt). The touches are younger than A(nk-2) and older than B(nk-2): the counted vmcnt(4) at
K-step nk - 2 retires them one K-step after their issue; their destination VGPR stays live across the loop (pinned after
every barrier) so that nothing else is allocated to it while they are in flight."""
EDITS = [
    ("gemm_bf16.hip", '''    if (nk == 1) load_aux();
    for (int kt = 0; kt < nk; ++kt) {''', '''    if (nk == 1) load_aux();
    int touch_reg = 0;
    for (int kt = 0; kt < nk; ++kt) {'''),
    ("gemm_bf16.hip", '''        if (nk >= 2 && kt == nk - 2) load_aux();''', '''        if (nk >= 2 && kt == nk - 2) load_aux();
        if constexpr (EPI == VPF_EPI_BIAS_RESIDUAL && !PART) {
            asm volatile("" : "+v"(touch_reg));
            if (kt == nk - 3) {
                // wave (wm, wn)'s residual slice: rows m0 + wm*128 + r, 128 B at column n0 + wn*64; lane: rows lane, lane + 64
                const int ln = opaque_lane();
                const int ra = min(m0 + wm * 128 + ln, M - 1), rb = min(m0 + wm * 128 + ln + 64, M - 1);
                const int c = min(n0 + wn * 64, N - 64);
                const bf16_t* p0 = residual + (int64_t)ra * ldc + c;
                const bf16_t* p1 = residual + (int64_t)rb * ldc + c;
                asm volatile("global_load_dword %0, %1, off\\n\\tglobal_load_dword %0, %2, off"
                             : "+v"(touch_reg) : "v"(p0), "v"(p1));
            }
        }'''),
]
