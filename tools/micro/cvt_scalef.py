"""Probe v_cvt_scalef32_pk_fp8_bf16 against the MX quantiser's element rule (tools/micro/cvt_scalef.hip).

For random bf16 pairs and every block exponent E in [-127, 125] the element bytes RNE(x * 2^-E) of mx8_pack8 are
compared with the scaled conversion given scale = 2^E and scale = 2^-E. Inputs are drawn so that |x| * 2^-E <= 448
(the quantiser's E never saturates). Prints the mismatch count per variant.
usage (GPU box): python tools/micro/cvt_scalef.py
"""
import ctypes
import os
import subprocess

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libcvtscalef.so")
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", SO,
                os.path.join(HERE, "cvt_scalef.hip")], check=True)
L = ctypes.CDLL(SO)
L.probe.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]


def main():
    rng = np.random.default_rng(0)
    n = 1 << 20
    E = rng.integers(-127, 126, n).astype(np.int32)
    # |x| = m * 2^(E + k), m in [1, 2), k in [-12, 7] (448 = 1.75 * 2^8): zeros, subnormal fp8 results, max values
    k = rng.integers(-12, 8, (n, 2))
    m = 1 + rng.random((n, 2))
    x = m * np.exp2(E[:, None] + k) * np.where(rng.random((n, 2)) < 0.5, -1, 1)
    x[rng.random((n, 2)) < 0.01] = 0.0
    xb = torch.from_numpy(x.astype(np.float32)).to(torch.bfloat16)
    xb = torch.where(xb.float().abs() * torch.exp2(-torch.from_numpy(E).float())[:, None] > 448,
                     torch.zeros_like(xb), xb)
    w = xb.view(torch.int16).numpy().astype(np.uint16).astype(np.uint32)
    packed = (w[:, 0] | (w[:, 1] << 16)).astype(np.uint32)
    din = torch.from_numpy(packed.view(np.int32)).cuda()
    de = torch.from_numpy(E).cuda()
    for variant, name in ((0, "scale = 2^E"), (1, "scale = 2^-E")):
        out = torch.zeros(n, dtype=torch.int32, device="cuda")
        assert L.probe(din.data_ptr(), de.data_ptr(), out.data_ptr(), n, variant) == 0
        o = out.cpu().numpy().view(np.uint32)
        ref, got = o & 0xffff, o >> 16
        bad = int((ref != got).sum())
        print(f"{name}: {bad} of {n} pairs differ" + (f" (e.g. in {packed[ref != got][:4]} E {E[ref != got][:4]} ref "
                                                      f"{ref[ref != got][:4]} got {got[ref != got][:4]})" if bad else ""))


if __name__ == "__main__":
    main()
