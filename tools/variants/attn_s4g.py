"""k_attn_stream, strip kinds in separate loops: 1 chunk per group, 5 groups resident (40 KiB), 4 waves per SIMD,
attn_step_pl: True (tools/variants/_attn_split.py)."""
import os
import runpy
EDITS = runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_attn_split.py"))["edits"](1, 5, 4, True)
