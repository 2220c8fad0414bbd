"""CPU: host logic — config surface, host Philox / resample planning vs the oracle, and the C-ABI library
(loads, exports every symbol include/vpf.h declares). No compute calls (no GPU here)."""
import ctypes
import os
import re

import numpy as np
import pytest

from oracle import pf
from vitparticlefiltertracker_amd import config as C
from vitparticlefiltertracker_amd import particle_filter as PF

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def test_config_defaults_and_yaml(tmp_path):
    d = C.load_config()
    assert d["model"]["arch"] == "vit_base_patch16_224" and d["particles"]["num"] == 4096
    p = tmp_path / "c.yaml"
    p.write_text("model: {arch: vit_tiny_patch16_224, dtype: fp32}\nparticles: {num: 256}\n")
    d = C.load_config(str(p))
    assert d["model"]["arch"] == "vit_tiny_patch16_224" and d["model"]["dtype"] == "fp32"
    assert d["particles"]["num"] == 256 and d["particles"]["seed"] == 1234       # merged defaults
    with pytest.raises(ValueError):
        C.load_config({"model": {"arch": "resnet50"}})
    with pytest.raises(ValueError):
        C.load_config({"resample": {"method": "multinomial"}})


def test_repo_config_yaml_loads():
    d = C.load_config(os.path.join(ROOT, "config.yaml"))
    assert d["model"]["arch"] in C.ARCHS


def test_arch_flops():
    assert abs(C.ARCHS["vit_base_patch16_224"].gflop_per_crop() - 35.126) < 0.01
    assert abs(C.ARCHS["vit_tiny_patch16_224"].gflop_per_crop() - 2.507) < 0.01
    assert abs(C.ARCHS["vit_large_patch14_336"].gflop_per_crop() - 381.918) < 0.05
    assert C.ARCHS["vit_large_patch14_336"].patch_kp == 640
    # executed work (the CLS-pruned last block): ViT-B loses one block's 2.908 GFLOP, keeps 0.021 of it
    b = C.ARCHS["vit_base_patch16_224"]
    assert abs(b.gflop_per_crop_executed(True) - 32.2396) < 1e-3
    assert b.gflop_per_crop_executed(False) > b.gflop_per_crop_executed(True)
    assert b.gflop_per_crop() - b.gflop_per_crop_executed(False) > 2.0


def test_host_philox_matches_oracle():
    rng = np.random.default_rng(0)
    for _ in range(200):
        ctr = [int(v) for v in rng.integers(0, 2 ** 32, 4)]
        key = [int(v) for v in rng.integers(0, 2 ** 32, 2)]
        assert PF.philox4x32_10(ctr, key) == [int(v) for v in pf.philox4x32_10(ctr, key)]
    for seed, frame in [(1234, 1), (0, 7), (2 ** 63 + 5, 99)]:
        assert PF.resample_word(seed, frame) == pf.resample_U(seed, frame)


def test_host_position_and_ranges():
    rng = np.random.default_rng(1)
    for _ in range(100):
        P = int(rng.integers(1, 5000))
        T = int(rng.integers(1, 1 << 56))
        U = int(rng.integers(0, 2 ** 32))
        for j in (0, P // 3, P - 1):
            assert PF.position(j, T, P, U) == pf.position(j, T, P, U)
    # ranges tile [0, P) in rank order
    P, G = 1000, 4
    Q = rng.integers(0, 1 << 40, P, dtype=np.int64)
    st = [(int(Q[r * 250:(r + 1) * 250].sum()), 0, 0, 0) for r in range(G)]
    _, T, offs, ranges = PF.plan_resample(st, P, 250, 12345)
    assert ranges[0][0] == 0 and ranges[-1][1] == P
    assert all(ranges[r][1] == ranges[r + 1][0] for r in range(G - 1))
    # uniform fallback
    uni, T, offs, ranges = PF.plan_resample([(0, 0, 0, 0)] * G, P, 250, 7)
    assert uni and T == P and ranges == [(0, 250), (250, 500), (500, 750), (750, 1000)]


def _declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "vpf.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(vpf_\w+)\(", hdr, re.M)))


def test_libvpf_exports_every_declared_symbol():
    from vitparticlefiltertracker_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    names = _declared_symbols()
    assert len(names) >= 17
    L = ctypes.CDLL(_lib.LIB_PATH)
    for n in names:
        assert hasattr(L, n), n
    assert set(names) - {"vpf_version"} == set(_lib.SIGNATURES)
    L.vpf_version.restype = ctypes.c_char_p
    assert b"gfx950" in L.vpf_version()


def test_libvpf_code_object_is_gfx950():
    from vitparticlefiltertracker_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_ops_refuse_cpu_tensors():
    """The product ops have no CPU implementation: calling them with CPU tensors must raise."""
    import torch
    from vitparticlefiltertracker_amd import ops  # noqa: F401
    p = torch.zeros(3, 4)
    with pytest.raises(Exception):
        torch.ops.vpf.predict_(p, 0, 1, 1, [1.0, 1.0, 0.1], 10.0, 10.0, [0.5, 2.0])


def test_config_template_update_range():
    from vitparticlefiltertracker_amd.config import load_config
    assert load_config(None)["likelihood"]["template_update"] == 0.0
    assert load_config({"likelihood": {"template_update": 0.25}})["likelihood"]["template_update"] == 0.25
    with pytest.raises(ValueError, match="template_update"):
        load_config({"likelihood": {"template_update": 1.5}})
    assert load_config({"model": {"dtype": "fp8"}})["model"]["dtype"] == "fp8"
    with pytest.raises(ValueError, match="dtype"):
        load_config({"model": {"dtype": "int4"}})


def test_config_rejects_bad_lambda():
    """SPEC S5: lambda must be finite and >= 0, otherwise w = exp(lam (sim - 1)) can exceed 1 and break the
    K + ceil(log2 P) <= 62 budget of the exact int64 resample."""
    from vitparticlefiltertracker_amd.config import load_config
    from vitparticlefiltertracker_amd.particle_filter import ParticleFilter
    assert load_config({"likelihood": {"lambda": 0.0}})["likelihood"]["lambda"] == 0.0
    for bad in (-1.0, float("nan"), float("inf")):
        with pytest.raises(ValueError, match="lambda"):
            load_config({"likelihood": {"lambda": bad}})
        with pytest.raises(ValueError, match="lam"):
            ParticleFilter(16, lam=bad, device="cpu")


def test_oracle_weights_clamp_and_nonfinite():
    """Oracle side of the SPEC S5 guards: sim > 1 is clamped (Q = 2^K exactly), NaN / inf give Q = 0."""
    import numpy as np
    from oracle import pf
    sim = np.array([1.0, 1.0000001, 1.5, np.nan, np.inf, -np.inf, 0.5, 0.9], np.float32)
    q = pf.weights_to_Q(sim, 20.0, 40)
    assert q[0] == q[1] == q[2] == 2 ** 40
    assert q[3] == q[4] == q[5] == 0
    assert 0 < q[6] < q[7] < 2 ** 40


def test_c_abi_rejects_bad_shapes_before_any_launch():
    """The C-ABI validates shapes on the host and returns VPF_ERR_ARG (-1) without touching the device (this
    runs without a GPU): the device-resident estimate/resample and the split-K GEMM."""
    from vitparticlefiltertracker_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    L = _lib.lib()
    fake = 4096                                          # never dereferenced: validation fails first
    er = L.vpf_estimate_resample
    # P = 0; P not a multiple of the shard; slot range past P; shard strides too short for several shards
    assert er(fake, 8, fake, 8, 24, 8, 0, 1, 1, 0, 0, fake, fake, 8, fake, fake, None) == -1
    assert er(fake, 8, fake, 8, 24, 7, 16, 1, 1, 0, 8, fake, fake, 8, fake, fake, None) == -1
    assert er(fake, 8, fake, 8, 24, 8, 16, 1, 1, 8, 17, fake, fake, 9, fake, fake, None) == -1
    assert er(fake, 4, fake, 8, 24, 8, 16, 1, 1, 0, 8, fake, fake, 8, fake, fake, None) == -1
    assert er(fake, 8, fake, 8, 20, 8, 16, 1, 1, 0, 8, fake, fake, 8, fake, fake, None) == -1
    sk = L.vpf_gemm_bf16_splitk
    # K = 768 not a multiple of 64 * 5 splits; workspace too small; LN without row statistics
    assert sk(fake, 768, fake, fake, None, None, None, fake, 768, 4, 768, 768, 0, 5, None, fake, 10 ** 7, None) == -1
    assert sk(fake, 768, fake, fake, None, None, None, fake, 768, 4, 768, 768, 0, 3, None, fake, 100, None) == -1
    assert sk(fake, 768, fake, fake, None, None, None, fake, 768, 4, 768, 768, 4, 3, None, fake, 10 ** 7, None) == -1
    sc = L.vpf_stats_combine
    # (round 5) no planes; a plane stride shorter than the rows; a misaligned output; D = 0
    assert sc(fake, 0, 100, 100, 768, 1e-6, fake, None) == -1
    assert sc(fake, 12, 99, 100, 768, 1e-6, fake, None) == -1
    assert sc(fake, 12, 100, 100, 768, 1e-6, fake + 4, None) == -1
    assert sc(fake, 12, 100, 100, 0, 1e-6, fake, None) == -1
    cr = L.vpf_crop_patches_bf16
    norm = (ctypes.c_float * 6)(*([0.5] * 6))
    # S not a multiple of the patch; Kp below 3 patch^2; Kp not a multiple of 8
    assert cr(fake, 224, 224, fake, fake, 8, 8, 64.0, 64.0, 224, 15, 768, norm, fake, None) == -1
    assert cr(fake, 224, 224, fake, fake, 8, 8, 64.0, 64.0, 224, 16, 760, norm, fake, None) == -1
    assert cr(fake, 336, 336, fake, fake, 8, 8, 64.0, 64.0, 336, 14, 590, norm, fake, None) == -1


def test_checkpoint_paths_round_trip():
    """the per-rank file save_checkpoint returns is accepted by load_checkpoint as is (no second suffix),
    and so is the base path, for one rank and for several."""
    from vitparticlefiltertracker_amd.tracker import Tracker
    t = Tracker.__new__(Tracker)              # host logic only: no device state needed
    for rank, world, base, want in ((0, 1, "ck", "ck.npz"), (0, 1, "ck.npz", "ck.npz"),
                                    (2, 4, "ck", "ck.rank2of4.npz"), (2, 4, "ck.rank2of4.npz", "ck.rank2of4.npz")):
        t.rank, t.world_size = rank, world
        f = t._checkpoint_file(base)
        assert f == want and t._checkpoint_file(f) == f


def test_product_library_has_no_knobs():
    """the product libvpf.so holds only the kernels it dispatches and reads no environment variable.
    * it imports no getenv (so VPF_GEMM_KERNEL=3, VPF_ATTN_TAIL16=0, VPF_MX8_VARIANT, VPF_CROP_LDS, ... cannot change
      a product launch: nothing reads them);
    * none of the lab kernels (persistent / four-wave GEMMs, the attention's software-pipelined strip) is in its code
      object; they live in the lab build (tools/gemm_lab);
    * vpf_gemm_tune accepts only the two product bf16 kernels (1, 5) and 0 (the per-shape defaults)."""
    import subprocess
    from vitparticlefiltertracker_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    dyn = subprocess.run(["nm", "-D", "--undefined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    assert "getenv" not in dyn and "secure_getenv" not in dyn, dyn
    blob = open(_lib.LIB_PATH, "rb").read()
    for lab_kernel in (b"k_gemm_pt", b"k_gemm_w4", b"attn_qk32", b"attn_sm_pv32", b"k_crop_patches_fast",
                       b"k_attn_bf16_ring"):
        assert lab_kernel not in blob, lab_kernel
    for product_kernel in (b"k_gemm_bf16", b"k_gemm_pp", b"k_gemm_mx8", b"k_attn_bf16_pipe", b"k_crop_patches_lds"):
        assert product_kernel in blob, product_kernel
    L = _lib.lib()
    try:
        for k in (2, 3, 4, 6, 7, 8, 9, 10, 13, 16, 17, 18, 20, 24, 27, 28, -2):
            assert L.vpf_gemm_tune(k, -1) == -1, k
        for k in (1, 5):
            assert L.vpf_gemm_tune(k, -1) == 0
        assert L.vpf_gemm_tune(1, 999) == -1
    finally:
        assert L.vpf_gemm_tune(0, -1) == 0


def test_weights_digest_tracks_the_weight_set():
    """the checkpoint fingerprint's weights_crc32 depends on the tensors, not on the configured seed."""
    from vitparticlefiltertracker_amd.config import ARCHS
    from vitparticlefiltertracker_amd.tracker import weights_digest
    from vitparticlefiltertracker_amd.weights import make_vit_weights
    a = ARCHS["vit_tiny_patch16_224"]
    d0, d0b, d1 = (weights_digest(make_vit_weights(a, seed=s)) for s in (0, 0, 1))
    assert d0 == d0b and d0 != d1
    w = make_vit_weights(a, seed=0)
    w["blocks.3.mlp.fc1.bias"] = w["blocks.3.mlp.fc1.bias"].clone()
    w["blocks.3.mlp.fc1.bias"][7] += 1e-3
    assert weights_digest(w) != d0


def test_fp8_frame_flop_split():
    """bench.py's fp8 frame fraction weighs the MX8 GEMMs' FLOPs against the fp8 peak: QKV, FC1, FC2 and
    (N <= 256) proj of blocks 0..L-2 run on MX8; the rest of the executed FLOPs stays bf16."""
    from vitparticlefiltertracker_amd.config import ARCHS
    b = ARCHS["vit_base_patch16_224"]
    N, D, F = b.tokens, b.dim, b.mlp
    assert abs(b.gflop_per_crop_mx8() - 2 * 11 * (3 * N * D * D + N * D * D + 2 * N * D * F) / 1e9) < 1e-9
    assert b.gflop_per_crop_mx8() < b.gflop_per_crop_executed() < b.gflop_per_crop()
    big = ARCHS["vit_large_patch14_336"]                 # N = 577: proj reads the bf16 attention output
    Nl, Dl, Fl = big.tokens, big.dim, big.mlp
    assert abs(big.gflop_per_crop_mx8() - 2 * 23 * (3 * Nl * Dl * Dl + 2 * Nl * Dl * Fl) / 1e9) < 1e-9


def test_product_sources_have_no_compile_time_knobs():
    """the product sources compile one form of each kernel. No preprocessor switch named VPF_* (the
    round-1..5 lab knobs: VPF_STREAM_WAVES, VPF_STREAM_LF, VPF_ATTN_VEARLY, VPF_ATTN_STREAM_MIN_N, VPF_CROP_LDS_DW) may
    select code in csrc/; A/B variants are text edits applied to a copy by tools/variant_lib.py."""
    csrc = os.path.join(ROOT, "vitparticlefiltertracker_amd", "csrc")
    bad = []
    for name in sorted(os.listdir(csrc)):
        if not name.endswith((".hip", ".h")):
            continue
        for i, line in enumerate(open(os.path.join(csrc, name)), 1):
            if re.match(r"\s*#\s*(if|ifdef|ifndef|elif)\b.*\bVPF_", line):
                bad.append(f"{name}:{i}: {line.strip()}")
    assert not bad, bad


def test_checkpoint_formats_are_refused_with_a_reason():
    """the weights' crc32 joined the fingerprint in round 4, so the format is now 3; format 1 files and
    format-2 files without the crc get an explicit 're-create the checkpoint' message instead of a generic
    configuration mismatch. ADVICE r5: a format-2 file that carries the crc (round 4 wrote it without a format bump) is
    checked like format 3, its crc included."""
    import json
    from vitparticlefiltertracker_amd.tracker import CHECKPOINT_FORMAT, _check_fingerprint
    assert CHECKPOINT_FORMAT == 3
    mine = {"arch": "vit_tiny_patch16_224", "weights_crc32": "0123abcd", "P": 16}
    cfg = np.array(json.dumps(mine))
    no_crc = np.array(json.dumps({k: v for k, v in mine.items() if k != "weights_crc32"}))
    _check_fingerprint({"format": np.int64(3), "config": cfg}, mine)
    _check_fingerprint({"format": np.int64(2), "config": cfg}, mine)
    with pytest.raises(ValueError, match="weights_crc32"):
        _check_fingerprint({"format": np.int64(2), "config": cfg}, {**mine, "weights_crc32": "ffffffff"})
    for fmt, c, words in ((1, cfg, "format 1"), (2, no_crc, "predates the weights' crc32")):
        with pytest.raises(ValueError, match=words):
            _check_fingerprint({"format": np.int64(fmt), "config": c}, mine)
    with pytest.raises(ValueError, match="weights_crc32"):
        _check_fingerprint({"format": np.int64(3), "config": cfg}, {**mine, "weights_crc32": "ffffffff"})
    with pytest.raises(ValueError, match="unknown"):
        _check_fingerprint({"format": np.int64(9), "config": cfg}, mine)


def _vregs(tok):
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"v(\d+)", tok)
    return {int(m.group(1))} if m else set()


def test_attention_q_loads_are_waited_before_any_use(tmp_path):
    """ADVICE r3 (Q-load asm safety), checked on the compiled code instead of trusted: the key-pipelined attention
    loads its Q fragments with inline-asm global_load_dwordx4 (hipcc must not count them, or it drains the K / V
    DMAs with them), so nothing but the kernel's own shape orders them before their uses. Rounds 2 and 4 each broke
    that shape once (a phi of asm outputs: register copies of not-yet-landed loads, NaNs on the GPU). Here the device
    code of csrc/attention.hip is compiled to gfx950 assembly and, for both k_attn_bf16_pipe instances and the
    key-streamed N > 256 kernel k_attn_stream (since round 6 also one load set for both strip kinds):
    * the Q loads are exactly four asm global_load_dwordx4 into VGPRs;
    * between the last of them and the empty pin asm that follows the counted wait, there is at least one
      `s_waitcnt vmcnt` and no instruction names any VGPR those loads write (no copy, no read, no reuse)."""
    import shutil
    import subprocess
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    src = os.path.join(ROOT, "vitparticlefiltertracker_amd", "csrc", "attention.hip")
    out = tmp_path / "attention.s"
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-Wno-unused-function", "--cuda-device-only",
                    "-S", "-o", str(out), src], check=True, capture_output=True)
    funcs = re.split(r"\n(?=_Z\S*:)", out.read_text())
    checked = 0
    for f in funcs:
        name = f.split(":", 1)[0]
        if not name.startswith("_Z"):     # the module header before the first kernel (it names them in .globl lines)
            continue
        if "k_attn_bf16_pipe" not in name and "k_attn_stream" not in name:
            continue
        L = [ln.strip() for ln in f.splitlines()]
        loads = [(i, _vregs(ln.split()[1].rstrip(","))) for i, ln in enumerate(L)
                 if ln.startswith("global_load_dwordx4 v[") and L[i - 1] == ";;#ASMSTART"]
        assert len(loads) == 4, (name, loads)
        last = loads[-1][0]
        pin = next(i for i in range(last + 1, len(L) - 1) if L[i] == ";;#ASMSTART" and L[i + 1] == ";;#ASMEND")
        assert any(L[i].startswith("s_waitcnt") and "vmcnt" in L[i] for i in range(last, pin)), name
        qregs = set().union(*(r for _, r in loads))
        touched = [L[i] for i in range(last + 1, pin)
                   if any(_vregs(t) & qregs for t in re.findall(r"v\[\d+:\d+\]|\bv\d+\b", L[i]))]
        assert not touched, (name, touched[:4])
        checked += 1
    assert checked == 3, checked


def test_attention_bf16_and_mx8_instances_share_the_step_form(tmp_path):
    """the MX8-output attention (fp8 path) must equal quantize_mx8 of the bf16-output attention bit for
    bit (tests/test_gpu_mx8.py), which holds only while both k_attn_bf16_pipe instances run the same 32-query step
    arithmetic. Round 5's red GPU run (gpurun_out/r5b, 3 x 197 x 12) came from a tree in which the N <= 256 kernel's
    32-query strips ran attn_step_lf (l summed from the bf16 probabilities on 4x4x4 MFMAs): the bf16 instance computes
    queries 192..196 on the 16-query strip (fp32 l), the MX8 instance, which has no 16-query strip, on the 32-query
    strip (then bf16-probability l), and the 3-bit e4m3 rounding exposed the difference. Checked on the compiled gfx950
    code: neither instance contains a 4x4x4 MFMA (the lf step form), and both carry the same number of 32x32x16 MFMAs
    (the same 32-query steps); only the bf16 instance has the 16-query strip's 16x16x32 MFMAs."""
    import collections
    import shutil
    import subprocess
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    src = os.path.join(ROOT, "vitparticlefiltertracker_amd", "csrc", "attention.hip")
    out = tmp_path / "attention.s"
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-Wno-unused-function", "--cuda-device-only",
                    "-S", "-o", str(out), src], check=True, capture_output=True)
    counts = {}
    for f in re.split(r"\n(?=_Z\S*:)", out.read_text()):
        name = f.split(":", 1)[0]
        if name.startswith("_Z") and "k_attn_bf16_pipe" in name:
            out8 = "Lb1E" in name
            counts[out8] = collections.Counter(ln.split()[0] for ln in map(str.strip, f.splitlines())
                                               if ln.startswith("v_mfma"))
    assert set(counts) == {False, True}, counts
    for c in counts.values():
        assert not any(k.startswith("v_mfma_f32_4x4x4") for k in c), counts
    assert counts[False]["v_mfma_f32_32x32x16_bf16"] == counts[True]["v_mfma_f32_32x32x16_bf16"] > 0, counts
    assert counts[False]["v_mfma_f32_16x16x32_bf16"] > 0 and counts[True]["v_mfma_f32_16x16x32_bf16"] == 0, counts


def test_config_bboxes_validation():
    """input.bboxes (several targets, main.py -> MultiTracker): null by default, else a non-empty list of [x, y, w, h]
    boxes with w, h > 0."""
    assert C.load_config(None)["input"]["bboxes"] is None
    c = C.load_config({"input": {"bboxes": [[1, 2, 30, 40], [5, 6, 7, 8]]}})
    assert c["input"]["bboxes"] == [[1, 2, 30, 40], [5, 6, 7, 8]]
    for bad in ([], [[1, 2, 3]], [[1, 2, 0, 4]], [[1, 2, 3, float("nan")]], "x"):
        with pytest.raises(ValueError):
            C.load_config({"input": {"bboxes": bad}})


def test_attention_kernels_fit_their_occupancy_without_spills(tmp_path):
    """The attention kernels' residency is a design parameter: k_attn_bf16_pipe runs two
    8-wave workgroups per CU and k_attn_stream (round 6) four 4-wave workgroups, i.e. four waves per SIMD, which holds
    only at <= 128 VGPRs (+ AGPRs) and, for k_attn_stream, <= 40 KiB of LDS per workgroup. A register spill would also
    put scratch loads, and the vmcnt waits that retire them, between the K / V DMA pieces and their counted waits.
    Checked on the compiled gfx950 code: no scratch, the register count and the static LDS size within those bounds."""
    import shutil
    import subprocess
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    src = os.path.join(ROOT, "vitparticlefiltertracker_amd", "csrc", "attention.hip")
    out = tmp_path / "attention.s"
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-Wno-unused-function", "--cuda-device-only",
                    "-S", "-o", str(out), src], check=True, capture_output=True)
    text = out.read_text()
    seen = set()
    for m in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", text, re.S):
        name, desc = m.group(1), m.group(2)
        kind = "stream" if "k_attn_stream" in name else "pipe" if "k_attn_bf16_pipe" in name else None
        if kind is None:
            continue
        field = {k: int(v) for k, v in re.findall(r"\.amdhsa_(\w+) (\d+)", desc)}
        assert field["private_segment_fixed_size"] == 0, (name, "scratch")
        assert field["next_free_vgpr"] <= 128, (name, field["next_free_vgpr"])
        if kind == "stream":
            assert field["group_segment_fixed_size"] <= 40 * 1024, (name, field["group_segment_fixed_size"])
        body = re.search(r"^" + re.escape(name) + r":(.*?)\.Lfunc_end", text, re.S | re.M).group(1)
        assert "scratch_" not in body, name
        seen.add(kind)
    assert seen == {"stream", "pipe"}, seen
