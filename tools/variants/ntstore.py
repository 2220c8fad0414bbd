"""GEMM bf16 output stores with the non-temporal hint (global_store_dwordx4 ... nt) in the pipelined-image and direct
epilogues: the C tiles (QKV 3.7 GB, FC1 5.0 GB per launch) are consumed by the next kernel from HBM anyway, so they
need not displace the A / W panels the other tiles of the XCD re-read from L2 (FC1 fetches 4.6x the A
panel)."""
_HELPER = '''// logical tile id -> output tile origin (the grouped order described above)'''
EDITS = [
    ("gemm_common.h", _HELPER, '''typedef unsigned u32x4_nt __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16_nt(void* p, uint4 v) {
    __builtin_nontemporal_store(u32x4_nt{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4_nt*>(p));
}
''' + _HELPER),
    ("gemm_common.h", "            if (ok) *reinterpret_cast<uint4*>(Cl + (int64_t)(i * 16 + h) * ldc) = v;",
     "            if (ok) st16_nt(Cl + (int64_t)(i * 16 + h) * ldc, v);"),
    ("gemm_common.h",
     "                *reinterpret_cast<uint4*>(Cl + (int64_t)(i * 16) * ldc + h * 32) = make_uint4(o[0], o[1], o[2], o[3]);",
     "                st16_nt(Cl + (int64_t)(i * 16) * ldc + h * 32, make_uint4(o[0], o[1], o[2], o[3]));"),
]
