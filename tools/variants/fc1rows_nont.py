"""(NT = False) FC1's direct-store epilogue (store_wave_tile_direct) with whole-row stores: lanes fr and fr ^ 8 swap a 16-B half
row through one DPP row_ror:8 per dword (4 v_cndmask + 4 DPP moves + 8 v_cndmask per 16-row group), so each store
instruction covers 8 whole 128-B rows instead of 16 half rows; NT = True also gives those stores the nt hint (which
only paid on whole-row stores: profiles/r6_lab/gemm_ntstore_ab.txt vs gemm_ntpipe_ab.txt)."""
NT = False
_OLD = '''        const int m = m0 + wm * 128 + i * 16 + fr;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint32_t o[4];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int j = 2 * h + k;
                f32x2 v01, v23;
                const f32x2 a01 = {acc[j][i][0], acc[j][i][1]}, a23 = {acc[j][i][2], acc[j][i][3]};
                const f32x2 b01 = {bv[j].x, bv[j].y}, b23 = {bv[j].z, bv[j].w};
                if constexpr (LN) {
                    const f32x2 c01 = {cv[j].x, cv[j].y}, c23 = {cv[j].z, cv[j].w};
                    v01 = __builtin_elementwise_fma(rsx, a01, __builtin_elementwise_fma(rsy, c01, b01));
                    v23 = __builtin_elementwise_fma(rsx, a23, __builtin_elementwise_fma(rsy, c23, b23));
                } else {
                    v01 = a01 + b01;
                    v23 = a23 + b23;
                }
                v01 = gelu_sig2(v01);
                v23 = gelu_sig2(v23);
                o[2 * k] = pack_bf2(v01.x, v01.y);
                o[2 * k + 1] = pack_bf2(v23.x, v23.y);
            }
            const int n = n0 + wn * 64 + h * 32 + fq * 8;
            if (m < M && n < N)
                *reinterpret_cast<uint4*>(Cl + (int64_t)(i * 16) * ldc + h * 32) = make_uint4(o[0], o[1], o[2], o[3]);
        }'''
_NEW = '''        uint32_t o[2][4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int j = 2 * h + k;
                f32x2 v01, v23;
                const f32x2 a01 = {acc[j][i][0], acc[j][i][1]}, a23 = {acc[j][i][2], acc[j][i][3]};
                const f32x2 b01 = {bv[j].x, bv[j].y}, b23 = {bv[j].z, bv[j].w};
                if constexpr (LN) {
                    const f32x2 c01 = {cv[j].x, cv[j].y}, c23 = {cv[j].z, cv[j].w};
                    v01 = __builtin_elementwise_fma(rsx, a01, __builtin_elementwise_fma(rsy, c01, b01));
                    v23 = __builtin_elementwise_fma(rsx, a23, __builtin_elementwise_fma(rsy, c23, b23));
                } else {
                    v01 = a01 + b01;
                    v23 = a23 + b23;
                }
                v01 = gelu_sig2(v01);
                v23 = gelu_sig2(v23);
                o[h][2 * k] = pack_bf2(v01.x, v01.y);
                o[h][2 * k + 1] = pack_bf2(v23.x, v23.y);
            }
        }
        {
            // lane fr < 8 (lo) keeps its h = 0 half of row fr and sends h = 1; lane fr ^ 8 keeps h = 1 of row fr | 8 and
            // sends h = 0: store 1 = rows i*16 + 0..7, store 2 = rows i*16 + 8..15, 8 lanes x 16 B per row each
            const bool lo = fr < 8;
            uint32_t rcv[4], d1[4], d2[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t snd = lo ? o[1][e] : o[0][e];
                rcv[e] = (uint32_t)__builtin_amdgcn_mov_dpp((int)snd, 0x128, 0xF, 0xF, false);   // row_ror:8
                d1[e] = lo ? o[0][e] : rcv[e];
                d2[e] = lo ? rcv[e] : o[1][e];
            }
            const int n = n0 + wn * 64 + (lo ? 0 : 32) + fq * 8;
            const int r1 = m0 + wm * 128 + i * 16 + (fr & 7);
            bf16_t* p1 = Cw + (int64_t)(i * 16) * ldc;
            if (r1 < M && n < N) STORE16(p1, make_uint4(d1[0], d1[1], d1[2], d1[3]));
            if (r1 + 8 < M && n < N) STORE16(p1 + (int64_t)8 * ldc, make_uint4(d2[0], d2[1], d2[2], d2[3]));
        }'''
EDITS = [
    ("gemm_common.h", _OLD, _NEW),
    ("gemm_common.h", '''    bf16_t* Cl = C + (int64_t)(m0 + wm * 128 + fr) * ldc + (n0 + wn * 64 + fq * 8);
    float4 bv[4], cv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = (wn * 64 + (j >> 1) * 32 + fq * 8 + (j & 1) * 4) * 4;''',
     '''    // whole-row stores: lane fr writes row fr & 7 (then + 8) at column half (fr < 8 ? 0 : 32)
    bf16_t* Cw = C + (int64_t)(m0 + wm * 128 + (fr & 7)) * ldc + (n0 + wn * 64 + (fr < 8 ? 0 : 32) + fq * 8);
    float4 bv[4], cv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = (wn * 64 + (j >> 1) * 32 + fq * 8 + (j & 1) * 4) * 4;'''),
]
DEFINES = ["-DSTORE16(p,v)=" + ("st16_nt((p),(v))" if NT else "(*reinterpret_cast<uint4*>(p)=(v))")]
