"""PROBE (wrong outputs by design): the residual epilogue's per-dword bf16 unpack / fp32 add / repack replaced by one
XOR with the residual dword (the residual loads and their data dependency kept), to price the residual arithmetic of
proj / FC2 before building an fp32-add form."""
EDITS = [("gemm_common.h",
          '''#pragma unroll
                for (int e = 0; e < 4; ++e)
                    o[e] = pack_bf2(bf2f((bf16_t)(w[e] & 0xffff)) + bf2f((bf16_t)(rr[e] & 0xffff)),
                                    bf2f((bf16_t)(w[e] >> 16)) + bf2f((bf16_t)(rr[e] >> 16)));
                v = make_uint4(o[0], o[1], o[2], o[3]);
                if (stats_out != nullptr) {   // wave-uniform; as store_wave_tile: the lane's partial back into its row''',
          '''#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] = w[e] ^ rr[e];
                v = make_uint4(o[0], o[1], o[2], o[3]);
                if (stats_out != nullptr) {   // wave-uniform; as store_wave_tile: the lane's partial back into its row''')]
