"""k_attn_stream, strip kinds in separate loops: 2 chunk(s) per group, 2 groups resident, 4 waves per SIMD,
attn_step_pl: True (tools/variants/_attn_split.py)."""
import os
import runpy
EDITS = runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_attn_split.py"))["edits"](2, 2, 4, True)
