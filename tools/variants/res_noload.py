"""PROBE (wrong outputs by design): the residual epilogue without its residual loads (zeros instead), to price the
residual read (128 KiB per tile, issued right after the K loop) in proj / FC2."""
EDITS = [("gemm_common.h",
          '''        res[it] = (m < M && n < N) ? *reinterpret_cast<const uint4*>(rl + (int64_t)roff * ldc) : make_uint4(0, 0, 0, 0);''',
          '''        res[it] = make_uint4((uint32_t)m & 1, 0, 0, (uint32_t)(int64_t)rl & 1);''')]
