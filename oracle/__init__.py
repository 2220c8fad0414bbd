"""ORACLE — TEST INFRASTRUCTURE ONLY (the checker, never the product).

A CPU restatement of the per-frame tracking path pinned by /root/repo/SPEC.md:

* `oracle.pf`  — ctypes binding of `pf_oracle.c` (Philox, predict, crop+im2col, estimate, exact
  integer systematic resample), bit-reproducible scalar C.
* `oracle.vit` — pure PyTorch-CPU fp32 functional ViT (timm/HF pre-norm semantics).
* `oracle.mx8` — numpy MX-fp8 format (e4m3fn round-half-even encoding, block exponents, scale planes,
  float64 GEMM on dequantised operands) for the fp8 path (configs[4]); pinned by the OCP value table and
  torch's float8_e4m3fn cast (tests/test_oracle_mx8.py).
* `oracle.tracker` — `OracleTracker`, the CPU mirror of `Tracker` used for end-to-end parity and as
  bench.py's `cpu_baseline` ("port" kind: the reference has no runnable code, README.md:1-63).

Pinning: the ViT is checked against `transformers.ViTModel` golden vectors (tests/golden/,
generated in the build container by tests/golden/make_golden.py); Philox against the published
Random123 known-answer vectors; predict/crop/resample against hand-computed known-answer tests. The
reference itself ships no tests or fixtures (README.md:54), so no reference-produced vector exists.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package.
"""
