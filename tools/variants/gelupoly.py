"""GELU without transcendentals in the GEMM epilogues (bf16 and MX8): x * Phi(x) with Phi(x) = 0.5 + xc P(xc^2),
xc = med3(x, -3.95, 3.95), P of degree 6 (IRLS minimax fit to the exact-erf GELU; max |error| 1.65e-4 over [-30, 30]
evaluated in fp32, against gelu_sig2's 2.7e-4): 2 v_med3_f32 + 9 packed ops per pair instead of 5 packed ops +
2 v_exp_f32 + 2 v_rcp_f32."""
_OLD = '''__device__ __forceinline__ f32x2 gelu_sig2(f32x2 x) {
    constexpr float L2E = 1.4426950408889634f;
    constexpr float c1 = -1.6003141571059616f * L2E, c2 = -0.06940178687219423f * L2E;
    const f32x2 q = (x * x) * c2 + c1;
    const f32x2 t = x * q;
    const f32x2 d = f32x2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + 1.0f;
    return x * f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}'''
_NEW = '''__device__ __forceinline__ f32x2 gelu_sig2(f32x2 x) {
    const f32x2 xc = {__builtin_amdgcn_fmed3f(x.x, -3.95f, 3.95f), __builtin_amdgcn_fmed3f(x.y, -3.95f, 3.95f)};
    const f32x2 t = xc * xc;
    f32x2 p = t * 2.4467887425627698e-08f + -1.6827345798038389e-06f;
    p = p * t + 4.9582135956441276e-05f;
    p = p * t + -0.0008293195880916253f;
    p = p * t + 0.008844213414175182f;
    p = p * t + -0.06472544825074197f;
    p = p * t + 0.3979885181252769f;
    return x * (xc * p + 0.5f);
}'''
EDITS = [("gemm_common.h", _OLD, _NEW)]
