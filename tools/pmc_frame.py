"""MFMA utilisation of every kernel of a bench run from one rocprofv3 --pmc pass ("rocprofv3 MFMA-busy
and HBM-bytes counters for one frame"; the HBM bytes are tools/pmc_traffic.py's two passes).

Counters (one pass: 2 SQ + 1 GRBM, within the per-pass limits of MI355X_MICROARCH.md §rocprofv3):
  SQ_VALU_MFMA_BUSY_CYCLES  MFMA-pipe busy cycles summed over the chip's 1024 SIMDs (= 16 per v_mfma_f32_16x16x32_bf16)
  GRBM_GUI_ACTIVE           GPU-active cycles summed over the 8 XCDs
  SQ_BUSY_CYCLES            (reported only)
Per dispatch: clock = GRBM_GUI_ACTIVE / 8 / wall (the DVFS-lowered clock the kernel ran at),
mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / 1024 / (GRBM_GUI_ACTIVE / 8) (fraction of the SIMD-cycles the MFMA pipes were busy).
mfma_busy x clock / 2.4 GHz is then the fraction of the 2.5 PF dense bf16 peak (quoted at 2.4 GHz) the kernel delivered.

    python tools/pmc_frame.py <pmc dir> [--frames F]     (F = frames in the run, for the per-frame ms column)
"""
import argparse
import collections
import csv
import glob
import os
import re

SIMDS, XCDS, PEAK_GHZ = 1024, 8, 2.4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--frames", type=float, default=1.0)
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.pmc_dir, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {a.pmc_dir}")
    disp = collections.defaultdict(dict)   # dispatch id -> {counter: value, name, grid, ms}
    for r in csv.DictReader(open(files[0])):
        d = disp[int(r["Dispatch_Id"])]
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        nm = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        d["name"] = re.sub(r"\(.*", "", nm)[:44]
        d["grid"] = int(r["Grid_Size"])
        d["ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    groups = collections.defaultdict(list)
    for d in disp.values():
        if "GRBM_GUI_ACTIVE" in d and "SQ_VALU_MFMA_BUSY_CYCLES" in d:
            groups[(d["name"], d["grid"])].append(d)
    tot_ms = sum(d["ms"] for g in groups.values() for d in g)
    tot_busy = sum(d["SQ_VALU_MFMA_BUSY_CYCLES"] for g in groups.values() for d in g) / SIMDS
    tot_cyc = sum(d["GRBM_GUI_ACTIVE"] for g in groups.values() for d in g) / XCDS
    print(f"{'kernel':44s} {'grid':>9s} {'n':>4s} {'ms/launch':>9s} {'ms/frame':>8s} {'GHz':>5s} "
          f"{'mfma_busy':>9s} {'of 2.5PF':>8s}")
    for key, g in sorted(groups.items(), key=lambda kv: -sum(d["ms"] for d in kv[1])):
        ms = sum(d["ms"] for d in g)
        cyc = sum(d["GRBM_GUI_ACTIVE"] for d in g) / XCDS
        busy = sum(d["SQ_VALU_MFMA_BUSY_CYCLES"] for d in g) / SIMDS / cyc if cyc else 0.0
        ghz = cyc / (ms * 1e6) if ms else 0.0
        if ms / tot_ms < 0.002:
            continue
        print(f"{key[0]:44s} {key[1]:9d} {len(g):4d} {ms / len(g):9.4f} {ms / a.frames:8.3f} {ghz:5.2f} "
              f"{busy:9.3f} {busy * ghz / PEAK_GHZ:8.3f}")
    ghz = tot_cyc / (tot_ms * 1e6)
    print(f"all kernels: {tot_ms / a.frames:.2f} ms per frame, {ghz:.2f} GHz average clock, MFMA busy "
          f"{tot_busy / tot_cyc:.3f} of the SIMD-cycles = {tot_busy / tot_cyc * ghz / PEAK_GHZ:.3f} of the 2.5 PF peak")


if __name__ == "__main__":
    main()
