"""VERDICT r5 #2's mapping for QKV / FC1: every column tile of one A row-panel on the same XCD, back to back (tile group
1: the XCD-contiguous logical ids of tile_of, then the A panel's column tiles consecutively), so an A panel is fetched
about once per XCD while the W panels (FC1: 12 x 384 KiB = 4.5 MiB, more than the XCD's 4 MiB L2) cycle through L2."""
EDITS = [("gemm_bf16.hip", "    return epilogue == VPF_EPI_LN_GELU ? 8 : kDefaultGroup;\n}",
          "    return (epilogue == VPF_EPI_LN_GELU || epilogue == VPF_EPI_LN) ? 1 : kDefaultGroup;\n}")]
