"""attn_p4 with the strip pair of a wave rotated by blockIdx % 4 (strips (w + b) % 4 and that + 4), so the co-resident
workgroups' light waves (N = 197: one wave has a single strip, one a strip and the 16-query strip) do not all land on
the same SIMD."""
import os
import runpy
_p4 = runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "attn_p4.py"))["EDITS"]
EDITS = [(f, o, n.replace("    const int sA = wid, sB = wid + 4;",
                          "    const int sA = (wid + (int)(blockIdx.x & 3)) & 3, sB = sA + 4;")) for f, o, n in _p4]
assert sum("blockIdx.x & 3" in n for _, _, n in EDITS) == 1
