"""As ntstore.py, but the nt hint only on the pipelined-image epilogue's stores (whole 128-B rows: QKV, proj, FC2, the
patch GEMM); FC1's direct stores (16 half rows per instruction) keep the default policy: round 6 session a measured nt
on every store as QKV -1.1 %, proj / FC2 level, FC1 +4.3 % (profiles/r6_lab/gemm_ntstore_ab.txt)."""
_HELPER = '''// logical tile id -> output tile origin (the grouped order described above)'''
EDITS = [
    ("gemm_common.h", _HELPER, '''typedef unsigned u32x4_nt __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16_nt(void* p, uint4 v) {
    __builtin_nontemporal_store(u32x4_nt{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4_nt*>(p));
}
''' + _HELPER),
    ("gemm_common.h", "            if (ok) *reinterpret_cast<uint4*>(Cl + (int64_t)(i * 16 + h) * ldc) = v;",
     "            if (ok) st16_nt(Cl + (int64_t)(i * 16 + h) * ldc, v);"),
]
