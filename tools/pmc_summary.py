"""Summarise rocprofv3 --pmc passes (tools/pmc_gemm.sh): for each pass directory, the counters of the libvpf kernels,
averaged over their dispatches (grouped by kernel and grid size), with the kernel time of each dispatch.
usage: python tools/pmc_summary.py <dir with pass subdirs> [kernel-name regex]"""
import collections
import csv
import glob
import os
import re
import sys

root = sys.argv[1]
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"k_gemm|k_attn")
res = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(dict)
for f in sorted(glob.glob(os.path.join(root, "*", "p_counter_collection.csv"))):
    pas = os.path.basename(os.path.dirname(f))
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if not pat.search(r["Kernel_Name"]):
                continue
            name = re.sub(r"\(.*", "", r["Kernel_Name"])[-60:]
            key = (name, int(r["Grid_Size"]))
            res[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[key][(pas, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
for key in sorted(res):
    d = list(dur[key].values())
    print(f"== {key[0]}  grid {key[1]}  dispatches {len(d)}  avg {sum(d) / len(d):.3f} ms")
    for c in sorted(res[key]):
        v = res[key][c]
        print(f"   {c:40s} {sum(v) / len(v):.4e}  (n={len(v)})")
