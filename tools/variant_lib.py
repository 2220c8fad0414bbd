"""Build an A/B variant of libvpf.so from the product sources plus a list of text replacements (design aid; the
product never loads it): tools/variants/<name>.py defines EDITS = [(file under csrc/, old, new), ...] (each `old` must
occur in the product file) and optionally DEFINES = ["-DX=1", ...]. The edited copy is compiled into
build/ab/<name>/ and linked as ab_libs/libvpf_<name>.so, which tools/lib_ab.py loads beside the product library
(outputs compared bit for bit) or bench.py loads through VPF_LIB_PATH. Since round 6 this replaces compile-time knobs in
the product sources (the product compiles one form of each kernel).

usage: python tools/variant_lib.py <name> [<name> ...]
"""
import os
import runpy
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "vitparticlefiltertracker_amd", "csrc")
SRCS = ["pf_kernels", "crop", "gemm_bf16", "gemm_mx8", "gemm_f32", "layernorm", "attention", "cls_attn"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-fvisibility=hidden"]


def build(name: str) -> str:
    spec = runpy.run_path(os.path.join(ROOT, "tools", "variants", f"{name}.py"))
    work = os.path.join(ROOT, "build", "ab", name)
    shutil.rmtree(work, ignore_errors=True)
    # same relative layout as the product (csrc/ next to ../../include/vpf.h)
    src = os.path.join(work, "pkg", "csrc")
    shutil.copytree(CSRC, src, ignore=shutil.ignore_patterns("*.o", "Makefile"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(work, "include"))
    for fname, old, new in spec["EDITS"]:
        p = os.path.join(src, fname)
        text = open(p).read()
        if text.count(old) != 1:
            raise SystemExit(f"variant {name}: edit target found {text.count(old)} times (need exactly 1) in {fname}: "
                             f"{old[:80]!r}")
        open(p, "w").write(text.replace(old, new))
    defines = list(spec.get("DEFINES", []))
    objs = [os.path.join(work, f"{s}.o") for s in SRCS]

    def cc(i):
        subprocess.run([HIPCC, *FLAGS, *defines, "-c", os.path.join(src, SRCS[i] + ".hip"), "-o", objs[i]], check=True)
    with ThreadPoolExecutor(max_workers=8) as ex:
        list(ex.map(cc, range(len(SRCS))))
    os.makedirs(os.path.join(ROOT, "ab_libs"), exist_ok=True)
    out = os.path.join(ROOT, "ab_libs", f"libvpf_{name}.so")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs], check=True)
    return out


if __name__ == "__main__":
    for n in sys.argv[1:]:
        print(build(n))
