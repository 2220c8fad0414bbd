"""k_attn_stream with 1 chunk(s) per group, 5 groups resident, 4 waves per SIMD (tools/variants/_attn_ring.py)."""
import os
import runpy
EDITS = runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_attn_ring.py"))["edits"](1, 5, 4)
