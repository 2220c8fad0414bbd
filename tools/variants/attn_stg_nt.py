"""N <= 256 attention (k_attn_bf16_pipe, bf16 output): the 32-query strips' output staged through a 2 KiB per-wave LDS
area and stored as whole 128-B rows (8 rows per store instruction instead of 32 rows x 32 B), in two 16-row passes;
cdna_hip_programming.md 'attack the per-BLOCK cost — O staged through LDS and stored as whole rows'. NT = True adds the
nt hint (whole-row stores took it well on the GEMMs: r6_lab/gemm_ntpipe_ab.txt)."""
NT = True
_OLD = '''        return;
    }
    if (q < q_rows) {
        bf16_t* orow = out + (row0 + q) * D + h * HD + 8 * hh;
#pragma unroll
        for (int k = 0; k < 4; ++k) *reinterpret_cast<uint4*>(orow + 16 * k) = ov[k];
    }
}'''
_NEW = '''        return;
    }
    {
        // lane (l32, hh) holds the 16-B chunks 2k + hh (dims 8c .. 8c+7) of query l32; chunk c of staged row r sits at
        // r * 128 + ((c ^ ((r >> 1) & 7)) << 4) (conflict-free for both the row-per-lane writes and the 8-lanes-per-row reads)
        char* stg = smem + 2 * NP * ROWB + wid * 2048;
        const int r16 = l32 & 15, half = l32 >> 4;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            if (half == p) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int c = 2 * k + hh;
                    *reinterpret_cast<uint4*>(stg + r16 * 128 + ((c ^ ((r16 >> 1) & 7)) << 4)) = ov[k];
                }
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int it = 0; it < 2; ++it) {
                const int r = it * 8 + (lane >> 3), c = lane & 7;
                const uint4 v = *reinterpret_cast<const uint4*>(stg + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
                const int qq = sid * 32 + 16 * p + r;
                if (qq < q_rows) STORE_O(out + (row0 + qq) * D + h * HD + 8 * c, v);
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}'''
EDITS = [
    ("attention.hip", _OLD, _NEW),
    ("attention.hip", '''        hipLaunchKernelGGL((k_attn_bf16_pipe<PIPE_CPB, false>), dim3((unsigned)(B * H)), dim3(512), lds,''',
     '''        hipLaunchKernelGGL((k_attn_bf16_pipe<PIPE_CPB, false>), dim3((unsigned)(B * H)), dim3(512), lds + 8 * 2048,'''),
]
DEFINES = ["-DSTORE_O(p,v)=" + ("__builtin_nontemporal_store(u32x4s{(v).x,(v).y,(v).z,(v).w},reinterpret_cast<u32x4s*>(p))" if NT else "(*reinterpret_cast<uint4*>(p)=(v))")]
if NT:
    EDITS.append(("attention.hip", "typedef float f32x16 __attribute__((ext_vector_type(16)));",
                  "typedef float f32x16 __attribute__((ext_vector_type(16)));\ntypedef unsigned u32x4s __attribute__((ext_vector_type(4)));"))
