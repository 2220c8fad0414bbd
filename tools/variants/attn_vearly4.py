"""The four-wave N > 256 attention (round 6 product) with round 5's early V^T reads back in attn_step_lf (issued right
after the QK^T MFMAs, retired by pv_mfmas' lgkmcnt(0)), plus a wait + pin of those reads at the entry of the rare
rescale branch, so that whatever the register allocator spills there holds landed values. At four waves per SIMD the
early reads spilled 11 VGPRs in that branch (tools/variants/attn_s4h.py, -7.2 % against the three-wave kernel, where
the late reads kept in the product gave -6.3 %)."""
import os
import subprocess

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
_old = subprocess.run(["git", "-C", _ROOT, "show", "fabd5ea:vitparticlefiltertracker_amd/csrc/attention.hip"],
                      capture_output=True, text=True, check=True).stdout
_i = _old.index("// pv32 split in two for the N > 256 kernel's steps (attn_step_lf)")
_j = _old.index("// The same step in the rounds 1-4 form (the N <= 256 kernel's)")
_PV = _old[_i:_j]
_f = "attention.hip"
EDITS = [
    (_f, "// The same step in the rounds 1-4 form (the N <= 256 kernel's)",
     _PV + "// The same step in the rounds 1-4 form (the N <= 256 kernel's)"),
    (_f, """    f32x16 s = qk32(Kt, lane, qf);
    mask(s);
    if (first) m = xor32_max(max16(s));""", """    f32x16 s = qk32(Kt, lane, qf);
    bf16x4 vr[2][2][2];
    pv_reads<2>(Vt, lane, vr);
    mask(s);
    if (first) m = xor32_max(max16(s));"""),
    (_f, """    if (!first && __builtin_expect(__any(!(ln[0] - lacc[0] <= 256.0f)), 0)) {
        f32x16 t = qk32(Kt, lane, qf);   // the scores again (s holds probabilities now)""",
     """    if (!first && __builtin_expect(__any(!(ln[0] - lacc[0] <= 256.0f)), 0)) {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vr[0][0][0]), "+v"(vr[0][0][1]), "+v"(vr[0][1][0]), "+v"(vr[0][1][1]),
                     "+v"(vr[1][0][0]), "+v"(vr[1][0][1]), "+v"(vr[1][1][0]), "+v"(vr[1][1][1])::"memory");
        f32x16 t = qk32(Kt, lane, qf);   // the scores again (s holds probabilities now)"""),
    (_f, """    lacc = ln;
    pv32<2>(Vt, lane, pf, o0, o1);
}

// The last key step when at most 8""", """    lacc = ln;
    pv_mfmas<2>(vr, pf, o0, o1);
}

// The last key step when at most 8"""),
]
