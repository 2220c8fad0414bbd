"""(Applies to the product before the round-6 four-wave k_attn_stream, i.e. up to commit fabd5ea.) Shared edits for
the N > 256 attention ring variants (attn_s4a/b/c, attn_s3r): k_attn_stream with CPB chunks per group, RING
groups resident and WPE waves per SIMD (the VGPR budget the compiler targets). The product is CPB = 2, RING = 3, WPE =
3 (48 KiB of LDS, three workgroups per CU). With RING groups resident, group g + RING - 1 is issued after group g's
barrier into group g - 1's slots (every wave has finished g - 1 there)."""


def edits(cpb: int, ring: int, wpe: int):
    f = "attention.hip"
    return [
        (f, "constexpr int STREAM_CPB = 2;", f"constexpr int STREAM_CPB = {cpb};"),
        (f, "constexpr int STREAM_RING = 3;", f"constexpr int STREAM_RING = {ring};"),
        (f, "__attribute__((amdgpu_waves_per_eu(3))) void k_attn_stream(",
         f"__attribute__((amdgpu_waves_per_eu({wpe}))) void k_attn_stream("),
        (f, "        const int issued = min(NG, max(STREAM_RING, g + 2));",
         "        const int issued = min(NG, max(STREAM_RING, g + STREAM_RING - 1));"),
        (f, "        if (g >= 1 && g + 2 < NG) issue_group(g + 2);",
         "        if (g >= 1 && g + STREAM_RING - 1 < NG) issue_group(g + STREAM_RING - 1);"),
    ]
