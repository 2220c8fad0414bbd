"""Per-launch HBM traffic of the ViT GEMMs from two rocprofv3 PMC passes over bench.py (one pass with
FETCH_SIZE, one with WRITE_SIZE: MI355X_MICROARCH.md §rocprofv3 PMC slots — they do not fit one pass).

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of a wide (16 B/lane)
streaming read, so fetch bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE (KiB) is exact for 16-B-per-lane stores.
Both count memory-side requests of the L2, Infinity-Cache hits included, i.e. an upper bound on HBM bytes.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> [--arch vit_base_patch16_224 --particles 4096 --dtype bf16]

Kernel naming: k_gemm_bf16<4> / k_gemm_pp<4> / k_gemm_mx8<4> = QKV (LN epilogue), <5> = FC1 (LN + GELU), <3> = patch embed, and
the two full-size <2> (bias + residual) launches of each block alternate proj, FC2 (dispatch order). CLS-row
launches (grid of one M tile) are skipped. --dtype fp8: the MX8 GEMMs' algorithmic bytes count e4m3 elements
(1 B) plus one e8m0 scale byte per 32 (configs[4]'s path: QKV / FC1 / FC2 / proj on MX8 operands).
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    rows = []
    for r in csv.DictReader(open(f[0])):
        if r["Counter_Name"] == counter:
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], int(r["Grid_Size"]), float(r["Counter_Value"])))
    rows.sort()
    return rows


def name_gemms(rows, min_grid):
    out, res_toggle = [], 0
    for _, kname, grid, val in rows:
        tag = next((t for t in ("k_gemm_bf16<", "k_gemm_pp<", "k_gemm_mx8<") if t in kname), None)
        if tag is None or grid < min_grid:
            continue
        epi = kname.split(tag)[1].split(">")[0].split(",")[0].strip()
        if epi == "4":
            n = "gemm_qkv"
        elif epi == "5":
            n = "gemm_fc1"
        elif epi == "3":
            n = "gemm_patch"
        elif epi == "2":
            n = "gemm_proj" if res_toggle == 0 else "gemm_fc2"
            res_toggle ^= 1
        else:
            continue
        out.append((n, val))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--arch", default="vit_base_patch16_224")
    ap.add_argument("--particles", type=int, default=4096)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"])
    ap.add_argument("--frame", default="224x224", help="the bench run's source frame HxW (recorded for the lookup)")
    a = ap.parse_args()
    from vitparticlefiltertracker_amd.config import ARCHS
    arch = ARCHS[a.arch]
    M = a.particles * arch.tokens
    min_grid = 512 * ((M + 255) // 256)          # at least one full column of tiles: skips CLS-row launches
    acc = defaultdict(lambda: {"fetch": [], "write": []})
    for n, v in name_gemms(load(a.fetch_dir, "FETCH_SIZE"), min_grid):
        acc[n]["fetch"].append(v)
    for n, v in name_gemms(load(a.write_dir, "WRITE_SIZE"), min_grid):
        acc[n]["write"].append(v)
    D, F = arch.dim, arch.mlp
    alg = {"gemm_qkv": (M * D + 3 * D * D + M * 3 * D) * 2, "gemm_proj": (M * D + D * D + 2 * M * D) * 2,
           "gemm_fc1": (M * D + F * D + M * F) * 2, "gemm_fc2": (M * F + F * D + 2 * M * D) * 2,
           "gemm_patch": (a.particles * arch.n_patches * (arch.patch_kp + D) + D * arch.patch_kp) * 2}
    if a.dtype == "fp8":
        q = 33 / 32                                   # e4m3 element + its share of the e8m0 scale
        # QKV: MX8 A, MX8 W, bf16 out; proj: MX8 A + W, bf16 residual in / out + the MX8 copy of h; FC1: MX8 in / W,
        # MX8 hidden out only; FC2: MX8 hidden + W, bf16 residual in / out + the MX8 copy of h
        alg.update({"gemm_qkv": (M * D + 3 * D * D) * q + M * 3 * D * 2,
                    "gemm_proj": (M * D + D * D) * q + 2 * M * D * 2 + M * D * q,
                    "gemm_fc1": (M * D + F * D + M * F) * q,
                    "gemm_fc2": (M * F + F * D) * q + 2 * M * D * 2 + M * D * q,
                    "gemm_patch": alg["gemm_patch"] + M * D * q})
        alg = {k: int(v) for k, v in alg.items()}
    res = {"arch": a.arch, "particles_per_gpu": a.particles, "dtype": a.dtype,
           "frame": [int(v) for v in a.frame.lower().split("x")],
           "note": "fetch = 2 x FETCH_SIZE (gfx950 wide-read correction), write = WRITE_SIZE; KiB -> bytes; "
                   "memory-side L2 requests (Infinity-Cache hits included)", "kernels": {}}
    for n, v in sorted(acc.items()):
        if not v["fetch"] or not v["write"]:
            continue
        fb = 2 * 1024 * sum(v["fetch"]) / len(v["fetch"])
        wb = 1024 * sum(v["write"]) / len(v["write"])
        res["kernels"][n] = {"launches": len(v["fetch"]), "fetch_bytes": round(fb), "write_bytes": round(wb),
                             "traffic_bytes": round(fb + wb), "algorithmic_bytes": alg.get(n),
                             "traffic_over_algorithmic": round((fb + wb) / alg[n], 3) if n in alg else None}
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
