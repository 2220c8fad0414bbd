"""The crop kernels' LDS window size in dwords (product: 10240 = 40 KiB, four workgroups per CU). Round 2's A/B
(profiles/r2_gemm_lab/crop_lds_window_ab.txt) was built by the retired tools/ab_libs.sh with -DVPF_CROP_LDS_DW; since
round 6 the product source holds no such knob and this edit builds the 80 KiB form (two workgroups per CU)."""
EDITS = [("crop.hip", "constexpr int CROP_LDS_DW = 10240;", "constexpr int CROP_LDS_DW = 20480;")]
