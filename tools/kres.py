"""Per-kernel VGPR / AGPR / spill / occupancy table from hipcc's kernel-resource-usage remarks.
usage: python tools/kres.py <file.hip> [name-filter-regex]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o",
                    "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
cur, rows = None, []
for line in r.stderr.splitlines():
    m = re.search(r"remark:\s+(.*?):\s*(.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for row in rows:
    if flt and not flt.search(row["name"]):
        continue
    print(f"{row.get('VGPRs', '?'):>4} vgpr {row.get('AGPRs', '?'):>4} agpr spill {row.get('VGPRs Spill', '?'):>3} "
          f"occ {row.get('Occupancy [waves/SIMD]', '?')}  {row['name'][:110]}")
