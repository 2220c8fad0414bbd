"""Read the operand maps of v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3) on the GPU (tools/micro/mx_probe.hip).

1. k pairing + A row map: A one-hot (lane la, byte ja) = 1.0; B byte jb of every lane = a value encoding jb
   (then: encoding lane >> 4). D's nonzero row = A's row of (la, ja); its value names the B (lane group, byte)
   holding the same k.
2. scale association: all-ones A / B, scale 2^0 everywhere except one lane's scale 2^1: which D entries grow and
   by how many K values.
3. op_sel: the same with the lane's 2^1 in byte 1 / 2 / 3 of its scale VGPR and op_sel = 1 / 2 / 3.
4. scale-k: which lane group's scale multiplies A element (lane, byte).
5. libvpf gemm_mx8 against float64 on uniform-scale and random data.
Findings (profiles/r1_gemm_lab/mx_probe.txt): A row = lane & 15, A / B symmetric; lane group g holds
K = 16g + j (bytes j < 16) and 64 + 16g + (j - 16) (bytes j >= 16); the scale of K-block b (32 values) is
lane group b's; op_sel = byte of the scale VGPR.
usage (GPU box): python tools/micro/mx_probe.py [maps]
"""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "libmxprobe.so"))
L.mx_probe.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
DEV = "cuda"
ONE = 0x38                                     # e4m3 1.0


def enc(j):                                    # 32 distinct exact e4m3 values (1 + m/8) 2^e
    return ((7 + j // 8) << 3) | (j % 8)


def dec(v):
    import math
    e = math.floor(math.log2(v))
    m = round((v / 2 ** e - 1) * 8)
    return e * 8 + m


def run(A, B, SA, SB, oa=0, ob=0):
    cfg = A.shape[0]
    D = torch.zeros(cfg, 64, 4, device=DEV)
    rc = L.mx_probe(A.data_ptr(), B.data_ptr(), SA.data_ptr(), SB.data_ptr(), D.data_ptr(), cfg, oa, ob,
                    torch.cuda.current_stream().cuda_stream)
    assert rc == 0, rc
    torch.cuda.synchronize()
    # assumed C/D map (shape-determined on gfx950): col = lane & 15, row = 4 (lane >> 4) + reg
    Dm = torch.zeros(cfg, 16, 16)
    Dc = D.cpu()
    for l in range(64):
        for r in range(4):
            Dm[:, 4 * (l >> 4) + r, l & 15] = Dc[:, l, r]
    return Dm


def probe_k():
    cfg = 64 * 32
    A = torch.zeros(cfg, 64, 32, dtype=torch.uint8)
    for la in range(64):
        for ja in range(32):
            A[la * 32 + ja, la, ja] = ONE
    S = torch.full((cfg, 64), 0x7F7F7F7F, dtype=torch.int32)
    res = {}
    for what in ("byte", "group"):
        B = torch.zeros(cfg, 64, 32, dtype=torch.uint8)
        for lb in range(64):
            for jb in range(32):
                B[:, lb, jb] = enc(jb if what == "byte" else lb >> 4)
        Dm = run(A.to(DEV), B.to(DEV), S.to(DEV), S.to(DEV))
        res[what] = Dm
    rows_ok, sym_ok, first_bad = 0, 0, []
    kmap = {}
    for la in range(64):
        for ja in range(32):
            c = la * 32 + ja
            Db = res["byte"][c]
            nz = (Db != 0).nonzero()
            rows = sorted(set(nz[:, 0].tolist()))
            if len(rows) != 1 or len(nz) != 16:
                first_bad.append((la, ja, rows, len(nz)))
                continue
            r = rows[0]
            jb = dec(Db[r, 0].item())
            gb = dec(res["group"][c][r, 0].item())
            kmap[(la, ja)] = (r, gb, jb)
            rows_ok += r == (la & 15)
            sym_ok += (gb, jb) == (la >> 4, ja)
    print(f"k probe: {len(kmap)} of 2048 single-row results; A row == lane&15: {rows_ok}; "
          f"B partner == (lane>>4, byte): {sym_ok}")
    if first_bad:
        print("  unexpected:", first_bad[:8])
    odd = [(k, v) for k, v in kmap.items() if v[0] != (k[0] & 15) or v[1:] != (k[0] >> 4, k[1])]
    print("  first asymmetric entries (la, ja) -> (row, B group, B byte):", odd[:16])


def probe_scale(which, byte=0):
    cfg = 64
    A = torch.full((cfg, 64, 32), ONE, dtype=torch.uint8)
    base = 0x7F7F7F7F
    SA = torch.full((cfg, 64), base, dtype=torch.int32)
    SB = torch.full((cfg, 64), base, dtype=torch.int32)
    T = SA if which == "A" else SB
    for ls in range(64):
        v = base & ~(0xFF << (8 * byte)) | (0x80 << (8 * byte))
        T[ls, ls] = v - (1 << 32) if v >= 2 ** 31 else v
    Dm = run(A.to(DEV), A.to(DEV), SA.to(DEV), SB.to(DEV), byte if which == "A" else 0, byte if which == "B" else 0)
    out = []
    for ls in range(64):
        inc = Dm[ls] - 128.0
        nz = (inc != 0).nonzero()
        rows = sorted(set(nz[:, 0].tolist()))
        cols = sorted(set(nz[:, 1].tolist()))
        out.append((ls, rows if len(rows) < 16 else "all", cols if len(cols) < 16 else "all",
                    sorted(set(inc[inc != 0].tolist()))))
    print(f"scale {which} byte {byte} (op_sel {byte}): lane -> rows, cols, increments")
    for o in out[:: 5]:
        print("  ", o)
    return out


def main_maps():
    probe_k()
    probe_scale("A")
    probe_scale("B")
    for b in (1, 2, 3):
        probe_scale("A", b)
    probe_scale("B", 1)


def probe_scale_k():
    """Which lane group's A scale multiplies A's element (lane la, byte ja): 4 configs per element."""
    cfg = 64 * 32 * 4
    A = torch.zeros(cfg, 64, 32, dtype=torch.uint8)
    SA = torch.full((cfg, 64), 0x7F7F7F7F, dtype=torch.int32)
    for la in range(64):
        for ja in range(32):
            for g in range(4):
                c = (la * 32 + ja) * 4 + g
                A[c, la, ja] = ONE
                SA[c, 16 * g: 16 * g + 16] = 0x80808080 - (1 << 32)
    B = torch.full((cfg, 64, 32), ONE, dtype=torch.uint8)
    SB = torch.full((cfg, 64), 0x7F7F7F7F, dtype=torch.int32)
    Dm = run(A.to(DEV), B.to(DEV), SA.to(DEV), SB.to(DEV))
    own, other = 0, []
    for la in range(64):
        for ja in range(32):
            gs = [g for g in range(4) if Dm[(la * 32 + ja) * 4 + g].abs().max().item() == 2.0]
            if gs == [la >> 4]:
                own += 1
            else:
                other.append((la, ja, gs))
    print(f"scale-k probe: elements scaled by their own lane group's scale: {own} / 2048; others: {other[:16]}")


def lib_uniform():
    """libvpf gemm_mx8 on data whose every block has the same scale byte, vs float64."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from vitparticlefiltertracker_amd import ops, _lib
    M, N, K = 512, 256, 256
    for name, gen in (("uniform-binade", lambda r, c: (torch.rand(r, c) + 1.0) * torch.sign(torch.randn(r, c))),
                      ("random", lambda r, c: torch.randn(r, c))):
        a = gen(M, K).to(torch.bfloat16).to(DEV)
        w = (gen(N, K) * 0.05).to(torch.bfloat16).to(DEV)
        a8, as8 = ops.mx8_empty(M, K, DEV)
        w8, ws8 = ops.mx8_empty(N, K, DEV)
        torch.ops.vpf.quantize_mx8_(a, 1, a8, as8)
        torch.ops.vpf.quantize_mx8_(w, 1, w8, ws8)
        A_ = ops.mx8_dequantize(a8, as8).double()
        W_ = ops.mx8_dequantize(w8, ws8).double()
        out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        torch.ops.vpf.gemm_mx8(a8, as8, w8, ws8, torch.zeros(N, device=DEV), None, None, None, _lib.VPF_EPI_BIAS, out)
        ref = A_ @ W_.t()
        err = (out.double() - ref).abs().max().item()
        sb = ops.mx8_scale_bytes(as8, M)
        print(f"lib {name}: max |err| {err:.4g} (ref max {ref.abs().max().item():.4g}); A scale bytes "
              f"{sb.min().item()}..{sb.max().item()}")


if __name__ == "__main__":
    import sys
    if "maps" in sys.argv:
        main_maps()
    probe_scale_k()
    lib_uniform()
