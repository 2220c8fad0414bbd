"""(Applies to the product before the round-6 four-wave k_attn_stream, i.e. up to commit fabd5ea; attn_s4i is that
form.) k_attn_stream with the two strip kinds in separate loops (attn_s3* / attn_s4* variants, round 6): the product
kept the 32-query strip's and the 16-query strip's registers (o0 / o1 / lacc and o16 / q16) live together through one chunk
loop; here one lambda, instantiated per strip kind, runs the group loop and the stores (the barrier schedule depends on
N only, as in k_attn_bf16_pipe), and one Q load set serves both kinds. The host adds a block when the 16-query strip
would otherwise share a wave with a 32-query strip (N % 32 in 1..16 and SF32 % 4 == 0). Parameters: CPB chunks per
group, RING groups resident, WPE waves per SIMD, PL: the 32-query step is attn_step_pl (True: fp32 l, the N <= 256
kernel's), attn_step_lf (False) or attn_step_lf with late V^T reads ("lfl")."""
import os

_SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                    "vitparticlefiltertracker_amd", "csrc", "attention.hip")


def _slice(text, start, end):
    i = text.index(start)
    j = text.index(end, i)
    return text[i:j]


_BODY = r'''    // one Q load set for both strip kinds (k_attn_bf16_pipe's rule: no branch between an asm load and its wait)
    bf16x8 qf[4];
    {
        const bf16_t* qp = act16 ? qbase + (int64_t)min(SF * 32 + (lane & 15), N - 1) * 3 * D + 8 * (lane >> 4)
                                 : qbase + (int64_t)min(st * 32 + l32, N - 1) * 3 * D + hh * 8;
        const int step = act16 ? 32 : 16;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
            asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qf[ks]) : "v"(qp + (act16 ? (ks & 1) : ks) * step));
    }
    auto issue_group = [&](int g) {
        int ln;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
        const int sub = ln >> 3, slot = ln & 7;
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
            const int pi = wid + WAVES * i;
            const int cc = pi >> 3, isv = (pi >> 2) & 1, j = pi & 3;
            const int c = g * STREAM_CPB + cc;
            const int r = c * 32 + 8 * j + sub;
            const int ch = isv ? (slot ^ (((r >> 1) & 1) << 2)) : (slot ^ ((r >> 1) & 7));
            const int sl = c % STREAM_SLOTS;
            __builtin_amdgcn_global_load_lds(
                (gptr_t)(qbase + (isv ? 2 * D : D) + (int64_t)min(r, N - 1) * 3 * D + ch * 8),
                (lptr_t)((isv ? Vs : Ks) + sl * 4096 + j * 1024), 16, 0, 0);
        }
    };
    const int g0 = min(NG, STREAM_RING);
    for (int g = 0; g < g0; ++g) issue_group(g);
    wait_vmcnt(PPW * g0);
    asm volatile("" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]) :: "memory");
    const int nfull = N >> 5;
    auto run_strip = [&](auto k16, bool act) {
        constexpr bool W16 = decltype(k16)::value;
        f32x16 o0 = {}, o1 = {};
        f32x4 lacc = {};
        (void)lacc;
        f32x4 o16[4] = {};
        float m = -INFINITY, l = 0.f;
        auto pin_q = [&]() {
            if constexpr (W16) asm volatile("" : "+v"(qf[0]), "+v"(qf[1]) :: "memory");
            else asm volatile("" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]) :: "memory");
        };
        for (int g = 0; g < NG; ++g) {
            const int issued = min(NG, max(STREAM_RING, g + STREAM_RING - 1));
            wait_vmcnt(PPW * (issued - g - 1));
            __builtin_amdgcn_s_barrier();
            pin_q();
            if (g >= 1 && g + STREAM_RING - 1 < NG) issue_group(g + STREAM_RING - 1);
            const int c_end = min((g + 1) * STREAM_CPB, nfull);
#pragma unroll 1
            for (int c = g * STREAM_CPB; c < c_end; ++c) {
                const int sl = c % STREAM_SLOTS;
                const char* Kt = Ks + sl * 4096;
                const char* Vt = Vs + sl * 4096;
                if (act) {
                    if constexpr (W16) attn_step16<false>(Kt, Vt, c * 32, N, lane, qf, scale_log2, m, l, o16);
                    else STEP32(false);
                }
            }
        }
        if (nfull < NT && act) {
            const int c = nfull, sl = c % STREAM_SLOTS;
            const char* Kt = Ks + sl * 4096;
            const char* Vt = Vs + sl * 4096;
            if constexpr (W16) attn_step16<true>(Kt, Vt, c * 32, N, lane, qf, scale_log2, m, l, o16);
            else if (N - c * 32 <= 8) TAIL8;
            else STEP32(true);
        }
        if (!act) return;
        if constexpr (W16) {
            const float inv = 1.0f / xor32_sum(xor16_sum(l));
            const int qq = SF * 32 + (lane & 15);
            if (qq < q_rows) {
                bf16_t* orow = out + (row0 + qq) * D + h * HD + 4 * (lane >> 4);
#pragma unroll
                for (int dt = 0; dt < 4; ++dt)
                    *reinterpret_cast<uint2*>(orow + 16 * dt) = make_uint2(pack_bf2(o16[dt][0] * inv, o16[dt][1] * inv),
                                                                          pack_bf2(o16[dt][2] * inv, o16[dt][3] * inv));
            }
        } else {
            const float inv = 1.0f / LSUM;
            uint32_t gx[8], gy[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const f32x16& o = k < 4 ? o0 : o1;
                const int b4 = 4 * (k & 3);
                gx[k] = pack_bf2(o[b4] * inv, o[b4 + 1] * inv);
                gy[k] = pack_bf2(o[b4 + 2] * inv, o[b4 + 3] * inv);
            }
            const int q = st * 32 + l32;
            uint4 ov[4];
#pragma unroll
            for (int k = 0; k < 8; k += 2) {
                const auto rx = __builtin_amdgcn_permlane32_swap(gx[k], gx[k + 1], false, false);
                const auto ry = __builtin_amdgcn_permlane32_swap(gy[k], gy[k + 1], false, false);
                ov[k >> 1] = make_uint4(rx[0], ry[0], rx[1], ry[1]);
            }
            if (q < q_rows) {
                bf16_t* orow = out + (row0 + q) * D + h * HD + 8 * hh;
#pragma unroll
                for (int k = 0; k < 4; ++k) *reinterpret_cast<uint4*>(orow + 16 * k) = ov[k];
            }
        }
    };
    if (act16) run_strip(std::true_type{}, true);
    else run_strip(std::false_type{}, act32);
}

'''


def edits(cpb: int, ring: int, wpe: int, pl: bool):
    f = "attention.hip"
    text = open(_SRC).read()
    old_body = _slice(text, "    // Q fragments by inline-asm loads, unconditionally for both strip kinds",
                      "// CLS-only attention (q_rows == 1")
    extra = []
    if pl == "lfl":   # attn_step_lf with the V^T reads after the softmax (pv32, as attn_step_pl): 16 VGPRs fewer live
        lf = _slice(text, "template <bool MASK>\n__device__ __forceinline__ void attn_step_lf(",
                    "// The last key step when at most 8")
        lfl = lf.replace("void attn_step_lf(", "void attn_step_lfl(").replace(
            "    bf16x4 vr[2][2][2];\n    pv_reads<2>(Vt, lane, vr);\n", "").replace(
            "    pv_mfmas<2>(vr, pf, o0, o1);", "    pv32<2>(Vt, lane, pf, o0, o1);")
        assert lfl.count("pv32<2>") == 1 and "pv_reads" not in lfl
        extra = [(f, "// The last key step when at most 8", lfl + "// The last key step when at most 8")]
    if pl is True:
        step = "attn_step_pl<M>(Kt, Vt, c * 32, N, lane, qf, scale_log2, m, l, o0, o1)"
        tail = "attn_step_tail8_pl(Kt, Vt, c * 32, N, lane, qf, scale_log2, m, l, o0, o1)"
        lsum = "xor32_sum(l)"
    else:
        step = ("attn_step_lfl" if pl == "lfl" else "attn_step_lf") + \
            "<M>(Kt, Vt, c * 32, N, lane, qf, scale_log2, c == 0, m, lacc, o0, o1)"
        tail = "attn_step_tail8_lf(Kt, Vt, c * 32, N, lane, qf, scale_log2, c == 0, m, lacc, o0, o1)"
        lsum = "xor32_sum(lacc[0])"
    body = _BODY.replace("STEP32(false)", step.replace("<M>", "<false>")).replace(
        "STEP32(true)", step.replace("<M>", "<true>")).replace("TAIL8", tail).replace("LSUM", lsum)
    return extra + [
        (f, "constexpr int STREAM_CPB = 2;", f"constexpr int STREAM_CPB = {cpb};"),
        (f, "constexpr int STREAM_RING = 3;", f"constexpr int STREAM_RING = {ring};"),
        (f, "__attribute__((amdgpu_waves_per_eu(3))) void k_attn_stream(",
         f"__attribute__((amdgpu_waves_per_eu({wpe}))) void k_attn_stream("),
        (f, old_body, body),
        (f, "    const int QB = need > W ? (need + W - 1) / W : 1;",
         "    const int t32 = N & 31;\n"
         "    const int need16 = need + (t32 >= 1 && t32 <= 16 && 32 * (N >> 5) < q_rows ? 1 : 0);\n"
         "    const int QB = need16 > W ? (need16 + W - 1) / W : 1;"),
    ]
