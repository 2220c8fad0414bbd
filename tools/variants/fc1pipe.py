"""FC1 (k_gemm_pp, EPI_LN_GELU) through the pipelined LDS-image epilogue, whose whole-row stores now carry the nt hint
(QKV -2.0 % with it), instead of the direct stores from the accumulators (round 4: direct -1.3 % against the image path
without nt)."""
EDITS = [("gemm_bf16.hip",
          "    constexpr bool DIRECT = (EPI == VPF_EPI_LN_GELU || EPI == VPF_EPI_BIAS_GELU) && !OUT8;\n",
          "    constexpr bool DIRECT = false;\n")]
