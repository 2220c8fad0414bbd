"""Summarise a rocprofv3 kernel_trace.csv per (kernel, grid size): calls and average duration, so the
full-size GEMM launches can be compared with bench.py's per-kernel HIP-event averages (the CLS-row launches
of the last block share the kernel name but not the grid).

    python tools/trace_by_grid.py <run_kernel_trace.csv>
"""
import csv
import sys
from collections import defaultdict

acc = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    acc[(name, int(r["Grid_Size_X"] if "Grid_Size_X" in r else r["Grid_Size"]))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
rows = sorted(acc.items(), key=lambda kv: -sum(kv[1]))
print(f"{'kernel':40s} {'grid':>10s} {'calls':>6s} {'avg_ms':>9s} {'total_ms':>9s}")
for (name, grid), v in rows:
    print(f"{name[:40]:40s} {grid:10d} {len(v):6d} {sum(v) / len(v):9.4f} {sum(v):9.2f}")
