"""GPU (MI355X): the ViT engine and the Tracker end to end against the CPU oracle.

* fp32 parity mode: CLS features within 1e-4 relative of oracle/vit.py; a full tracking clip keeps every
  per-frame (x, y, scale) within 1e-4 relative of OracleTracker (north_star tolerance).
* bf16 product mode: features close to the fp32 oracle (cosine >= 0.999, reported tolerance); with the GPU's
  own int64 weights injected into the oracle every frame, resample ancestors and particle states are
  bit-exact and the estimates agree to 1e-12.
"""
import numpy as np
import pytest
import torch

from oracle import pf
from oracle import vit as ovit
from oracle.tracker import OracleMultiTracker, OracleTracker
from vitparticlefiltertracker_amd.config import ARCHS, ViTArch, load_config
from vitparticlefiltertracker_amd.frames import synthetic_clip
from vitparticlefiltertracker_amd.weights import make_vit_weights

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _crops(arch, n, seed=0):
    rng = np.random.default_rng(seed)
    frame = rng.integers(0, 256, (224, 224, 3), dtype=np.uint8)
    p = np.empty((3, n), np.float32)
    p[0] = rng.uniform(40, 184, n); p[1] = rng.uniform(40, 184, n); p[2] = rng.uniform(0.6, 1.8, n)
    return frame, p


@pytest.mark.parametrize("name,dtype,n", [("vit_tiny_patch16_224", "fp32", 5), ("vit_tiny_patch16_224", "bf16", 9),
                                          ("vit_base_patch16_224", "bf16", 3), ("vit_base_patch16_224", "fp32", 2),
                                          ("vit_large_patch14_336", "bf16", 2), ("vit_large_patch14_336", "fp32", 1),
                                          ("vit_small_patch16_224", "fp8", 7), ("vit_base_patch16_224", "fp8", 3),
                                          ("vit_large_patch14_336", "fp8", 2)])
def test_vit_features_vs_oracle(name, dtype, n):
    from vitparticlefiltertracker_amd.vit import ViTEngine
    arch = ARCHS[name]
    w = make_vit_weights(arch, seed=4, perturb_affine=True)
    frame, p = _crops(arch, n)
    eng = ViTEngine(arch, w, dtype, DEV, n)
    feat = eng.features(torch.from_numpy(frame).to(DEV), torch.from_numpy(p).to(DEV), (64.0, 64.0)).double().cpu()
    patches = pf.crop_patches(frame, p, (64.0, 64.0), arch.img_size, arch.patch, arch.patch_kp, (0.5,) * 3, (0.5,) * 3)
    ref = ovit.features_from_patches(torch.from_numpy(patches), w, arch).double()
    if dtype == "fp32":
        torch.testing.assert_close(feat, ref, rtol=1e-4, atol=1e-4 * ref.abs().max().item())
    else:
        # bf16: >= 0.999; fp8 (MX e4m3 weights and GEMM inputs, configs[4]): reported tolerance >= 0.99
        cos = torch.nn.functional.cosine_similarity(feat, ref, dim=1)
        assert cos.min().item() > (0.999 if dtype == "bf16" else 0.99), cos


@pytest.mark.parametrize("name,dtype", [("vit_base_patch16_224", "bf16"), ("vit_small_patch16_224", "fp8"),
                                        ("vit_large_patch14_336", "bf16")])
def test_cls_fused_tail_equals_kv_path(name, dtype):
    """The last block's CLS attention without K / V (vpf_cls_attn_fold_bf16 between two block-diagonal GEMMs)
    against the K / V GEMM + attention path it replaces (ViTEngine(cls_fused=False)), and both against the fp32
    oracle."""
    from vitparticlefiltertracker_amd.vit import ViTEngine
    arch = ARCHS[name]
    w = make_vit_weights(arch, seed=6, perturb_affine=True)
    n = 33
    frame, p = _crops(arch, n, seed=2)
    fd, pd = torch.from_numpy(frame).to(DEV), torch.from_numpy(p).to(DEV)
    fused = ViTEngine(arch, w, dtype, DEV, n)
    assert fused.cls_fused
    f1 = fused.features(fd, pd, (64.0, 64.0)).double().cpu()
    plain = ViTEngine(arch, w, dtype, DEV, n, cls_fused=False)
    assert not plain.cls_fused
    f0 = plain.features(fd, pd, (64.0, 64.0)).double().cpu()
    cos = torch.nn.functional.cosine_similarity(f1, f0, dim=1)
    assert cos.min().item() > 0.9995, cos
    patches = pf.crop_patches(frame, p, (64.0, 64.0), arch.img_size, arch.patch, arch.patch_kp, (0.5,) * 3, (0.5,) * 3)
    ref = ovit.features_from_patches(torch.from_numpy(patches), w, arch).double()
    bar = 0.999 if dtype == "bf16" else 0.99
    assert torch.nn.functional.cosine_similarity(f1, ref, dim=1).min().item() > bar


def _tiny_cfg(P, dtype, arch="vit_tiny_patch16_224"):
    return load_config({"model": {"arch": arch, "dtype": dtype, "weights": {"seed": 3}},
                        "particles": {"num": P, "seed": 99}})


def test_fp8_rejects_unaligned_width():
    from vitparticlefiltertracker_amd.vit import ViTEngine
    arch = ARCHS["vit_tiny_patch16_224"]                  # D = 192: not a multiple of the 128-deep MX8 K-tile
    with pytest.raises(ValueError, match="fp8"):
        ViTEngine(arch, make_vit_weights(arch, seed=0), "fp8", DEV, 4)


@pytest.mark.parametrize("arch_name,P,frames", [("vit_tiny_patch16_224", 64, 6), ("vit_base_patch16_224", 64, 4),
                                                ("vit_base_patch16_224", 128, 3), ("vit_large_patch14_336", 6, 3)])
def test_tracker_fp32_matches_oracle_end_to_end(arch_name, P, frames):
    """north_star's state tolerance: per-frame (x, y, s) within 1e-4 relative of OracleTracker on identical frames,
    in the fp32 parity mode. ViT-B/16 is the metric's model; ViT-L/14 @ 336 is configs[3]'s
    (N = 577 tokens, D = 1024, 16 heads; 6 particles keep the CPU oracle's share to seconds)."""
    from vitparticlefiltertracker_amd import Tracker
    cfg = _tiny_cfg(P, "fp32", arch_name)
    arch = ARCHS[arch_name]
    w = make_vit_weights(arch, seed=3)
    clip = synthetic_clip(frames)
    tr = Tracker(cfg, weights=w)
    ot = OracleTracker(cfg, w, arch)
    tr.init(clip[0], (80, 80, 64, 64))
    ot.init(clip[0], (80, 80, 64, 64))
    torch.testing.assert_close(tr.template.double().cpu(), torch.from_numpy(ot.template).double(), rtol=1e-4, atol=1e-5)
    for f in clip[1:]:
        e_gpu = np.array(tr.track(f))
        e_ref = np.array(ot.track(f))
        np.testing.assert_allclose(e_gpu, e_ref, rtol=1e-4)


@pytest.mark.parametrize("use_graph,dtype,arch_name,P", [(True, "bf16", "vit_tiny_patch16_224", 256),
                                                          (False, "bf16", "vit_tiny_patch16_224", 256),
                                                          (True, "fp8", "vit_small_patch16_224", 256),
                                                          (True, "bf16", "vit_base_patch16_224", 1),
                                                          (True, "bf16", "vit_tiny_patch16_224", 37),
                                                          (True, "fp8", "vit_small_patch16_224", 3)])
def test_tracker_bf16_weight_injection_bit_exact(use_graph, dtype, arch_name, P):
    """Ragged sizes too: one particle (197 GEMM rows, a single partial tile everywhere), 37 and 3 (odd shard
    chunks, GEMM row counts that are not a multiple of the 256-row tile, CLS GEMMs of a few rows)."""
    from vitparticlefiltertracker_amd import Tracker
    cfg = _tiny_cfg(P, dtype, arch_name)
    arch = ARCHS[arch_name]
    w = make_vit_weights(arch, seed=3)
    clip = synthetic_clip(6)
    tr = Tracker(cfg, weights=w, use_graph=use_graph)
    ot = OracleTracker(cfg, w, arch)
    tr.init(clip[0], (80, 80, 64, 64))
    ot.init(clip[0], (80, 80, 64, 64))
    for k, f in enumerate(clip[1:], start=1):
        tr._upload(f)
        tr.frame_index += 1
        tr.pf.predict(tr.frame_index)
        tr.weigh()
        Q = tr.pf.Q.cpu().numpy().copy()
        e_gpu = tr.pf.estimate()
        anc = tr.pf.resample().cpu().numpy()
        e_ref = ot.track(f, Q=Q)                      # oracle predicts itself, then uses the GPU's weights
        assert np.array_equal(anc, ot.last_ancestors), f"frame {k}"
        assert np.array_equal(tr.pf.particles_soa.cpu().numpy().view(np.uint32), ot.particles.view(np.uint32))
        np.testing.assert_allclose(e_gpu, e_ref, rtol=1e-12)
        assert Q.sum() > 0


def test_configs0_32_frame_clip_matches_oracle():
    """BASELINE.json configs[0] as written: 256 particles, ViT-Ti/16, a 32-frame synthetic 224 x 224
    clip, run by the GPU Tracker (bf16, HIP-graph replay, the product's step(): estimate and resample in one device
    call) against OracleTracker with the GPU's int64 weights injected every frame. All 31 tracked frames: every
    ancestor and particle state bit-exact, the estimate within 1e-12 relative. Every 8th frame the bf16 CLS features of
    4 predicted particles are also checked against the fp32 oracle's (cosine >= 0.999)."""
    from vitparticlefiltertracker_amd import Tracker
    cfg = _tiny_cfg(256, "bf16")
    arch = ARCHS["vit_tiny_patch16_224"]
    w = make_vit_weights(arch, seed=3)
    clip = synthetic_clip(32)
    assert len(clip) == 32 and clip[0].shape == (224, 224, 3)
    tr = Tracker(cfg, weights=w)
    ot = OracleTracker(cfg, w, arch)
    tr.init(clip[0], (80, 80, 64, 64))
    ot.init(clip[0], (80, 80, 64, 64))
    for k, f in enumerate(clip[1:], start=1):
        tr._upload(f)
        tr.frame_index += 1
        tr.pf.predict(tr.frame_index)
        tr.weigh()
        Q = tr.pf.Q.cpu().numpy().copy()
        assert Q.sum() > 0, f"frame {k}"
        if k % 8 == 0:
            pred = tr.pf.particles_soa.cpu().numpy()
            tr.engine.weights_from_tokens(tr.n_local, tr.template, tr.lam, tr.bits, want_feat=True)
            idx = np.array([0, 85, 170, 255])
            feat = tr.engine.feat[idx.tolist()].double().cpu().numpy()
            ref_f = ot.features(f, np.ascontiguousarray(pred[:, idx])).astype(np.float64)
            cos = (feat * ref_f).sum(1) / (np.linalg.norm(feat, axis=1) * np.linalg.norm(ref_f, axis=1))
            assert cos.min() >= 0.999, (k, cos)
        e_gpu = tr.pf.step()
        e_ref = ot.track(f, Q=Q)
        assert np.array_equal(tr.pf.last_ancestors.cpu().numpy(), ot.last_ancestors), f"frame {k}: ancestors"
        assert np.array_equal(tr.pf.particles_soa.cpu().numpy().view(np.uint32), ot.particles.view(np.uint32)), k
        np.testing.assert_allclose(e_gpu, e_ref, rtol=1e-12)


def test_configs0_bf16_free_running_drift_vs_fp32_oracle():
    """VERDICT r5 (parity caveat): the bf16 product tracker FREE-RUNNING — its own bf16 weights decide every resample —
    against the fp32 CPU oracle free-running on the same configs[0] clip (256 particles, ViT-Ti/16, 32 frames; the same
    seeds, so the two differ only through the bf16 forward's weights). Once one int64 weight differs the two filters
    resample differently and their particle sets part, so this is a drift bound, not a parity bar: per frame the
    estimates' |dx|, |dy| <= 4 px and |ds| <= 0.05 (round 6, first run: 1.99 / 1.45 px, 0.013). The distance of each
    track from the target's true centre (frames.target_box) is reported, not asserted: with seeded random-init ViT
    weights (no checkpoint offline) the features do not single out the target, and the fp32 oracle stays near the
    start box exactly as the bf16 tracker does (both ~59 px behind the target by frame 31). The per-frame record goes
    to $VPF_TEST_REPORT_DIR/bf16_drift_configs0.json when that is set (profiles/r6_bf16_drift_configs0.json)."""
    import json
    import os

    from vitparticlefiltertracker_amd import Tracker
    from vitparticlefiltertracker_amd.frames import target_box
    cfg = _tiny_cfg(256, "bf16")
    arch = ARCHS["vit_tiny_patch16_224"]
    w = make_vit_weights(arch, seed=3)
    clip = synthetic_clip(32)
    bbox0 = (80, 80, 64, 64)
    tr = Tracker(cfg, weights=w)
    ot = OracleTracker(cfg, w, arch)                      # the fp32 CPU path (model.dtype is the GPU's only)
    tr.init(clip[0], bbox0)
    ot.init(clip[0], bbox0)
    rows = []
    for k, f in enumerate(clip[1:], start=1):
        g = np.array(tr.track(f), np.float64)
        r = np.array(ot.track(f), np.float64)
        x, y, bw, bh = target_box(k, bbox0, (2, 1))
        truth = np.array([x + 0.5 * bw, y + 0.5 * bh])
        rows.append({"frame": k, "bf16": g.tolist(), "fp32_oracle": r.tolist(), "drift": (g - r).tolist(),
                     "bf16_err_px": float(np.abs(g[:2] - truth).max()),
                     "fp32_err_px": float(np.abs(r[:2] - truth).max())})
    d = np.array([row["drift"] for row in rows])
    summary = {"max_abs_dx": float(np.abs(d[:, 0]).max()), "max_abs_dy": float(np.abs(d[:, 1]).max()),
               "max_abs_ds": float(np.abs(d[:, 2]).max()),
               "max_bf16_err_px": max(row["bf16_err_px"] for row in rows),
               "max_fp32_err_px": max(row["fp32_err_px"] for row in rows)}
    rep = os.environ.get("VPF_TEST_REPORT_DIR")
    if rep:
        os.makedirs(rep, exist_ok=True)
        with open(os.path.join(rep, "bf16_drift_configs0.json"), "w") as fh:
            json.dump({"workload": "configs[0]: 256 particles, vit_tiny_patch16_224, 32-frame synthetic 224x224 clip",
                       "summary": summary, "frames": rows}, fh, indent=1)
    assert summary["max_abs_dx"] <= 4.0 and summary["max_abs_dy"] <= 4.0 and summary["max_abs_ds"] <= 0.05, summary


@pytest.mark.parametrize("dtype,arch_name", [("bf16", "vit_tiny_patch16_224"), ("fp8", "vit_small_patch16_224")])
def test_tracker_graph_equals_eager(dtype, arch_name):
    from vitparticlefiltertracker_amd import Tracker
    cfg = _tiny_cfg(128, dtype, arch_name)
    w = make_vit_weights(ARCHS[arch_name], seed=3)
    clip = synthetic_clip(5)
    outs = []
    for g in (True, False):
        tr = Tracker(cfg, weights=w, use_graph=g)
        tr.init(clip[0], (80, 80, 64, 64))
        outs.append(tr.run(clip[1:]))
    assert np.array_equal(outs[0], outs[1])


def test_tracker_fp8_1080p_follows_target():
    """configs[4] geometry on one GPU at a small particle count: ViT-B/16 fp8, 1080x1920 source frames. The
    tracked centre stays on the moving target (it moves 2.2 px/frame; tolerance 24 px)."""
    from vitparticlefiltertracker_amd import Tracker
    from vitparticlefiltertracker_amd.frames import target_box
    cfg = load_config({"model": {"arch": "vit_base_patch16_224", "dtype": "fp8"},
                       "particles": {"num": 512, "seed": 5}})
    clip = synthetic_clip(6, 1080, 1920, bbox0=(900, 500, 64, 64))
    tr = Tracker(cfg)
    tr.init(clip[0], (900, 500, 64, 64))
    for k, f in enumerate(clip[1:], start=1):
        x, y, s = tr.track(f)
        bx, by, bw, bh = target_box(k, (900, 500, 64, 64))
        assert abs(x - (bx + bw / 2)) < 24 and abs(y - (by + bh / 2)) < 24, (k, x, y)


def test_main_reads_y4m_clip(tmp_path):
    """The reference's entry point end to end (README.md:37, 42): `main.py --config` with `input.source` a
    YUV4MPEG2 video, decoded on the prefetch thread into pinned buffers; the tracked positions (JSON) follow
    the target through the 4:2:0 colour round trip."""
    import json
    import sys
    import yaml
    from vitparticlefiltertracker_amd.frames import target_box, write_y4m
    sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
    import main as vpf_main
    clip = synthetic_clip(6)
    video = tmp_path / "clip.y4m"
    write_y4m(video, clip, chroma="420")
    cfg = {"model": {"arch": "vit_tiny_patch16_224", "dtype": "bf16"}, "particles": {"num": 256, "seed": 3},
           "input": {"source": str(video), "frames": 6, "bbox0": [80, 80, 64, 64]}}
    cpath = tmp_path / "config.yaml"
    cpath.write_text(yaml.safe_dump(cfg))
    out = tmp_path / "track.json"
    assert vpf_main.main(["--config", str(cpath), "--out", str(out)]) == 0
    res = json.loads(out.read_text())
    assert [r["frame"] for r in res] == [1, 2, 3, 4, 5]
    for r in res:
        bx, by, bw, bh = target_box(r["frame"])
        assert abs(r["x"] - (bx + bw / 2)) < 16 and abs(r["y"] - (by + bh / 2)) < 16, r


def test_template_update():
    """likelihood.template_update = alpha: the template moves toward the feature at the estimate and stays unit;
    alpha = 0 leaves it bit-identical."""
    from vitparticlefiltertracker_amd import Tracker
    clip = synthetic_clip(4)
    outs = {}
    for alpha in (0.0, 0.5):
        cfg = load_config({"model": {"arch": "vit_tiny_patch16_224", "dtype": "bf16"},
                           "particles": {"num": 128, "seed": 3}, "likelihood": {"template_update": alpha}})
        tr = Tracker(cfg)
        tr.init(clip[0], (80, 80, 64, 64))
        t0 = tr.template.clone()
        est = [tr.track(f) for f in clip[1:]]
        outs[alpha] = (t0, tr.template.clone(), est)
    t0, t1, _ = outs[0.0]
    assert torch.equal(t0, t1)
    t0, t1, est = outs[0.5]
    assert not torch.equal(t0, t1)
    assert abs(t1.norm().item() - 1.0) < 1e-5
    cos = torch.dot(t0, t1).item()
    assert 0.5 < cos < 1.0, cos
    for k, (x, y, s) in enumerate(est, start=1):     # still on the target
        assert abs(x - (80 + 2 * k + 32)) < 16 and abs(y - (80 + k + 32)) < 16


def test_main_video_out(tmp_path):
    """main.py --video-out writes every frame with the tracked box overlaid (a .y4m sink)."""
    import sys
    import yaml
    from vitparticlefiltertracker_amd.frames import read_y4m
    sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
    import main as vpf_main
    cfg = {"model": {"arch": "vit_tiny_patch16_224", "dtype": "bf16"}, "particles": {"num": 128, "seed": 3},
           "input": {"source": "synthetic", "frames": 4}}
    cpath = tmp_path / "config.yaml"
    cpath.write_text(yaml.safe_dump(cfg))
    vid = tmp_path / "out.y4m"
    assert vpf_main.main(["--config", str(cpath), "--video-out", str(vid)]) == 0
    frames = list(read_y4m(vid))
    assert len(frames) == 4 and frames[0].shape == (224, 224, 3)
    red = (frames[2][..., 0] > 200) & (frames[2][..., 1] < 60) & (frames[2][..., 2] < 60)
    assert red.sum() > 100                          # the box outline is there


def test_main_png_frames_in_and_out(tmp_path):
    """main.py on a directory of PNG frames (read through Pillow), writing PNG frames with --frame-format png: the
    positions equal those of the same clip given as a .npy file (PNG is lossless), and every output frame exists."""
    import json
    import sys
    import yaml
    from vitparticlefiltertracker_amd.frames import read_image_pil, synthetic_clip, write_image_pil
    sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
    import main as vpf_main
    clip = synthetic_clip(4)
    src = tmp_path / "png_in"
    src.mkdir()
    for k, f in enumerate(clip):
        write_image_pil(src / f"{k:03d}.png", f)
    np.save(tmp_path / "clip.npy", clip)
    outs = []
    for name, source in (("png", src), ("npy", tmp_path / "clip.npy")):
        cfg = {"model": {"arch": "vit_tiny_patch16_224", "dtype": "bf16"}, "particles": {"num": 64, "seed": 3},
               "input": {"source": str(source), "frames": 4}}
        cpath = tmp_path / f"{name}.yaml"
        cpath.write_text(yaml.safe_dump(cfg))
        o = tmp_path / f"{name}.json"
        argv = ["--config", str(cpath), "--out", str(o)]
        if name == "png":
            argv += ["--video-out", str(tmp_path / "png_out"), "--frame-format", "png"]
        assert vpf_main.main(argv) == 0
        outs.append(json.loads(o.read_text()))
    assert outs[0] == outs[1] and len(outs[0]) == 3
    written = sorted((tmp_path / "png_out").glob("frame_*.png"))
    assert len(written) == 4 and read_image_pil(written[0]).shape == (224, 224, 3)


def test_main_multi_object(tmp_path):
    """main.py with input.bboxes (README.md:46-50, SPEC S9): one MultiTracker over two targets; the JSON has one record
    per frame with both targets, target 0's track is main.py's single-target track bit for bit (the batched pass is
    row-independent and target 0 keeps particles.seed), and --video-out draws both boxes."""
    import json
    import sys
    import yaml
    from vitparticlefiltertracker_amd.frames import read_pnm
    sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
    import main as vpf_main
    base = {"model": {"arch": "vit_tiny_patch16_224", "dtype": "bf16"}, "particles": {"num": 128, "seed": 3},
            "input": {"source": "synthetic", "frames": 4, "bbox0": [80, 80, 64, 64]}}
    one, two = tmp_path / "one.yaml", tmp_path / "two.yaml"
    one.write_text(yaml.safe_dump(base))
    multi = {**base, "input": {**base["input"], "bboxes": [[80, 80, 64, 64], [20, 140, 48, 40]]}}
    two.write_text(yaml.safe_dump(multi))
    o1, o2, vid = tmp_path / "one.json", tmp_path / "two.json", tmp_path / "frames"
    assert vpf_main.main(["--config", str(one), "--out", str(o1)]) == 0
    assert vpf_main.main(["--config", str(two), "--out", str(o2), "--video-out", str(vid)]) == 0
    r1, r2 = json.loads(o1.read_text()), json.loads(o2.read_text())
    assert [r["frame"] for r in r2] == [1, 2, 3] and all(len(r["targets"]) == 2 for r in r2)
    for a, b in zip(r1, r2):
        assert (a["x"], a["y"], a["scale"]) == (b["targets"][0]["x"], b["targets"][0]["y"], b["targets"][0]["scale"])
    assert len(list(vid.glob("frame_*.ppm"))) == 4
    f0 = read_pnm(vid / "frame_00000.ppm")            # lossless sink: the outlines are exact (255, 0, 0)
    for x, y, w, h in multi["input"]["bboxes"]:
        assert (f0[y, x:x + w] == (255, 0, 0)).all() and (f0[y:y + h, x] == (255, 0, 0)).all()
        assert (f0[y + h - 1, x:x + w] == (255, 0, 0)).all() and (f0[y:y + h, x + w - 1] == (255, 0, 0)).all()
    # checkpoint after frame 2, resume for frame 3: the same positions as the uninterrupted run, bit for bit
    ck, o3 = tmp_path / "ck", tmp_path / "resumed.json"
    assert vpf_main.main(["--config", str(two), "--frames", "3", "--checkpoint", str(ck)]) == 0
    assert vpf_main.main(["--config", str(two), "--resume", str(ck) + ".npz", "--out", str(o3)]) == 0
    assert json.loads(o3.read_text()) == r2[2:]
    # a single-target tracker refuses a multi-target checkpoint
    with pytest.raises(ValueError):
        vpf_main.main(["--config", str(one), "--resume", str(ck) + ".npz"])


def test_multitracker_one_target_equals_tracker():
    """MultiTracker's batched pass is row-independent: with one target it reproduces Tracker bit for bit."""
    from vitparticlefiltertracker_amd import MultiTracker, Tracker
    cfg = _tiny_cfg(128, "bf16")
    w = make_vit_weights(ARCHS["vit_tiny_patch16_224"], seed=3)
    clip = synthetic_clip(5)
    tr = Tracker(cfg, weights=w)
    tr.init(clip[0], (80, 80, 64, 64))
    mt = MultiTracker(cfg, 1, weights=w)
    mt.init(clip[0], [(80, 80, 64, 64)])
    for f in clip[1:]:
        a = tr.track(f)
        (b,) = mt.track(f)
        assert a == b
    assert torch.equal(tr.pf.particles_soa, mt.pfs[0].particles_soa)


TWO_BOXES = [(40, 50, 48, 48), (200, 150, 64, 40)]


def _two_target_clip(frames):
    """Two textured targets with their own box sizes (48 x 48, 64 x 40) and trajectories on a 240 x 320 frame."""
    rng = np.random.default_rng(11)
    bg = rng.integers(0, 256, (240, 320, 3), dtype=np.uint8)
    tex = [np.random.default_rng(s).integers(0, 256, (h, w, 3), dtype=np.uint8) for s, (w, h) in
           ((21, (48, 48)), (22, (64, 40)))]
    starts, vel = [(40, 50), (200, 150)], [(3, 1), (-2, -2)]
    clip = []
    for t in range(frames):
        f = bg.copy()
        for k in range(2):
            x, y = starts[k][0] + vel[k][0] * t, starts[k][1] + vel[k][1] * t
            h, w = tex[k].shape[:2]
            f[y:y + h, x:x + w] = tex[k]
        clip.append(f)
    centres = [[(starts[k][0] + vel[k][0] * t + tex[k].shape[1] / 2, starts[k][1] + vel[k][1] * t + tex[k].shape[0] / 2)
                for k in range(2)] for t in range(frames)]
    return clip, centres


def test_multitracker_two_targets():
    """Two textured targets with their own box sizes and trajectories, tracked in one batched ViT pass."""
    from vitparticlefiltertracker_amd import MultiTracker
    clip, centres = _two_target_clip(6)
    cfg = load_config({"model": {"arch": "vit_tiny_patch16_224", "dtype": "bf16"},
                       "particles": {"num": 256, "seed": 7}})
    mt = MultiTracker(cfg, 2)
    mt.init(clip[0], TWO_BOXES)
    for t, f in enumerate(clip[1:], start=1):
        est = mt.track(f)
        for k, (x, y, s) in enumerate(est):
            cx, cy = centres[t][k]
            assert abs(x - cx) < 16 and abs(y - cy) < 16, (t, k, x, y, cx, cy)


# ------------------------------------------------------------- §8f rank 4 against the oracle (SPEC S9)
@pytest.mark.parametrize("arch_name,P,frames", [("vit_tiny_patch16_224", 64, 5), ("vit_base_patch16_224", 64, 3)])
def test_tracker_template_update_fp32_matches_oracle(arch_name, P, frames):
    """likelihood.template_update = 0.5 in the fp32 parity mode: per frame the estimate (x, y, s) is within 1e-4
    relative of OracleTracker's (north_star's state tolerance) and the updated template within 1e-4 of the oracle's
    S9 update (the crop at the estimate, its feature, the fp32 blend and renormalisation)."""
    from vitparticlefiltertracker_amd import Tracker
    cfg = load_config({"model": {"arch": arch_name, "dtype": "fp32", "weights": {"seed": 3}},
                       "particles": {"num": P, "seed": 99}, "likelihood": {"template_update": 0.5}})
    arch = ARCHS[arch_name]
    w = make_vit_weights(arch, seed=3)
    clip = synthetic_clip(frames)
    tr = Tracker(cfg, weights=w)
    ot = OracleTracker(cfg, w, arch)
    tr.init(clip[0], (80, 80, 64, 64))
    ot.init(clip[0], (80, 80, 64, 64))
    t0 = ot.template.copy()
    for k, f in enumerate(clip[1:], start=1):
        np.testing.assert_allclose(np.array(tr.track(f)), np.array(ot.track(f)), rtol=1e-4, err_msg=f"frame {k}")
        np.testing.assert_allclose(tr.template.cpu().numpy(), ot.template, rtol=1e-4, atol=1e-5,
                                   err_msg=f"frame {k}: template")
    assert float(np.dot(t0, ot.template)) < 0.99999      # the template did move


def test_tracker_template_update_bf16_q_injected():
    """bf16 product mode, template_update = 0.5: with the GPU's weights injected, every frame's ancestors and
    resampled states are bit-exact and the estimate agrees to 1e-12; the GPU's updated template (bf16 features) stays
    within cosine 0.999 of the oracle's fp32 S9 update at the same estimate."""
    from vitparticlefiltertracker_amd import Tracker
    cfg = load_config({"model": {"arch": "vit_tiny_patch16_224", "dtype": "bf16", "weights": {"seed": 3}},
                       "particles": {"num": 256, "seed": 99}, "likelihood": {"template_update": 0.5}})
    arch = ARCHS["vit_tiny_patch16_224"]
    w = make_vit_weights(arch, seed=3)
    clip = synthetic_clip(6)
    tr = Tracker(cfg, weights=w)
    ot = OracleTracker(cfg, w, arch)
    tr.init(clip[0], (80, 80, 64, 64))
    ot.init(clip[0], (80, 80, 64, 64))
    for k, f in enumerate(clip[1:], start=1):
        tr._upload(f)
        tr.frame_index += 1
        tr.pf.predict(tr.frame_index)
        tr.weigh()
        Q = tr.pf.Q.cpu().numpy().copy()
        est = tr.pf.step()
        tr.update_template(est)
        e_ref = ot.track(f, Q=Q)                       # oracle: predict, injected Q, estimate, resample, S9 update
        np.testing.assert_allclose(est, e_ref, rtol=1e-12)
        assert np.array_equal(tr.pf.last_ancestors.cpu().numpy(), ot.last_ancestors), f"frame {k}"
        assert np.array_equal(tr.pf.particles_soa.cpu().numpy().view(np.uint32), ot.particles.view(np.uint32))
        cos = float(np.dot(tr.template.cpu().numpy().astype(np.float64), ot.template.astype(np.float64)))
        assert cos > 0.999, (k, cos)


@pytest.mark.parametrize("alpha", [0.0, 0.5])
def test_multitracker_fp32_matches_oracle(alpha):
    """K = 2 targets with different box sizes (48 x 48, 64 x 40) in the fp32 parity mode: every target's estimate
    within 1e-4 relative of OracleMultiTracker's (each target cropped with its own box, weighed against its own
    template, its own particle seed), per frame; with a template update every target's template within 1e-4 of the
    oracle's. A wrong per-target box or template in the batched pass fails this."""
    from vitparticlefiltertracker_amd import MultiTracker
    clip, _ = _two_target_clip(5)
    cfg = load_config({"model": {"arch": "vit_tiny_patch16_224", "dtype": "fp32", "weights": {"seed": 3}},
                       "particles": {"num": 64, "seed": 7}, "likelihood": {"template_update": alpha}})
    arch = ARCHS["vit_tiny_patch16_224"]
    w = make_vit_weights(arch, seed=3)
    mt = MultiTracker(cfg, 2, weights=w)
    om = OracleMultiTracker(cfg, 2, w, arch)
    mt.init(clip[0], TWO_BOXES)
    om.init(clip[0], TWO_BOXES)
    for k in range(2):
        np.testing.assert_allclose(mt.templates[k].cpu().numpy(), om.targets[k].template, rtol=1e-4, atol=1e-5)
    for t, f in enumerate(clip[1:], start=1):
        e_gpu, e_ref = mt.track(f), om.track(f)
        for k in range(2):
            np.testing.assert_allclose(np.array(e_gpu[k]), np.array(e_ref[k]), rtol=1e-4, err_msg=f"frame {t} target {k}")
            np.testing.assert_allclose(mt.templates[k].cpu().numpy(), om.targets[k].template, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("alpha", [0.0, 0.5])
def test_multitracker_bf16_q_injected(alpha):
    """K = 2 targets, bf16 product mode: with each target's GPU weights injected into its oracle filter, every
    target's ancestors and resampled states are bit-exact and its estimate agrees to 1e-12, frame after frame
    (with a template update too: the GPU's templates within cosine 0.999 of the oracle's)."""
    from vitparticlefiltertracker_amd import MultiTracker
    clip, _ = _two_target_clip(6)
    cfg = load_config({"model": {"arch": "vit_tiny_patch16_224", "dtype": "bf16", "weights": {"seed": 3}},
                       "particles": {"num": 128, "seed": 7}, "likelihood": {"template_update": alpha}})
    arch = ARCHS["vit_tiny_patch16_224"]
    w = make_vit_weights(arch, seed=3)
    mt = MultiTracker(cfg, 2, weights=w)
    om = OracleMultiTracker(cfg, 2, w, arch)
    mt.init(clip[0], TWO_BOXES)
    om.init(clip[0], TWO_BOXES)
    for t, f in enumerate(clip[1:], start=1):
        mt._upload(f)
        mt.frame_index += 1
        for pf_ in mt.pfs:
            pf_.height, pf_.width = f.shape[0], f.shape[1]
            pf_.predict(mt.frame_index)
        mt.weigh()
        Qs = [pf_.Q.cpu().numpy().copy() for pf_ in mt.pfs]
        e_gpu = mt.step()
        e_ref = om.track(f, Qs)
        for k in range(2):
            np.testing.assert_allclose(e_gpu[k], e_ref[k], rtol=1e-12)
            assert np.array_equal(mt.pfs[k].last_ancestors.cpu().numpy(), om.targets[k].last_ancestors), (t, k)
            assert np.array_equal(mt.pfs[k].particles_soa.cpu().numpy().view(np.uint32),
                                  om.targets[k].particles.view(np.uint32)), (t, k)
            cos = float(np.dot(mt.templates[k].cpu().numpy().astype(np.float64),
                               om.targets[k].template.astype(np.float64)))
            assert cos > 0.999, (t, k, cos)
            assert Qs[k].sum() > 0


def test_tracker_upload_mixed_sources_and_size_change():
    """Frames may arrive as numpy arrays, pinned host tensors or device tensors in any order: the estimates
    equal an all-numpy run. A frame of another size afterwards re-bounds predict (particles stay inside the
    new frame) instead of clamping to the init frame."""
    from vitparticlefiltertracker_amd import Tracker
    cfg = _tiny_cfg(128, "bf16")
    w = make_vit_weights(ARCHS["vit_tiny_patch16_224"], seed=3)
    clip = synthetic_clip(6)
    ref = Tracker(cfg, weights=w)
    ref.init(clip[0], (80, 80, 64, 64))
    e_ref = [ref.track(f) for f in clip[1:]]
    tr = Tracker(cfg, weights=w)
    tr.init(torch.from_numpy(clip[0]).pin_memory(), (80, 80, 64, 64))
    srcs = [torch.from_numpy(clip[1]).pin_memory(), clip[2], torch.from_numpy(clip[3]).to(DEV), clip[4],
            torch.from_numpy(clip[5]).pin_memory()]
    assert [tr.track(f) for f in srcs] == e_ref
    big = np.random.default_rng(1).integers(0, 256, (300, 400, 3), dtype=np.uint8)
    big[:224, :224] = clip[5]
    tr.track(big)
    assert (tr.pf.height, tr.pf.width) == (300, 400)
    small = np.ascontiguousarray(clip[5][:100, :120])
    tr.track(small)
    assert (tr.pf.height, tr.pf.width) == (100, 120)
    p = tr.pf.particles_soa.cpu().numpy()
    assert p[0].max() <= 119 and p[1].max() <= 99 and p.min() >= 0


@pytest.mark.parametrize("alpha", [0.0, 0.5])
def test_checkpoint_resume_bit_exact(tmp_path, alpha):
    """SURVEY.md §5 checkpoint / resume: 3 frames, save_checkpoint, a NEW Tracker loads it and tracks frames 4-6:
    estimates, ancestors and particle states equal an uninterrupted run bit for bit (counter-based noise; with a
    template update the updated template travels in the checkpoint). A second uninterrupted run is also
    bit-identical to the first (the run-to-run determinism check that stands in for a race detector)."""
    from vitparticlefiltertracker_amd import Tracker
    cfg = load_config({"model": {"arch": "vit_tiny_patch16_224", "dtype": "bf16", "weights": {"seed": 3}},
                       "particles": {"num": 256, "seed": 99}, "likelihood": {"template_update": alpha}})
    w = make_vit_weights(ARCHS["vit_tiny_patch16_224"], seed=3)
    clip = synthetic_clip(7)

    def run(tr, frames):
        return [(tr.track(f), tr.pf.last_ancestors.cpu().numpy().copy(), tr.pf.particles_soa.cpu().numpy().copy())
                for f in frames]

    tr = Tracker(cfg, weights=w)
    tr.init(clip[0], (80, 80, 64, 64))
    ref = run(tr, clip[1:])
    tr = Tracker(cfg, weights=w)
    tr.init(clip[0], (80, 80, 64, 64))
    again = run(tr, clip[1:])
    a = Tracker(cfg, weights=w)
    a.init(clip[0], (80, 80, 64, 64))
    first = run(a, clip[1:4])
    path = a.save_checkpoint(str(tmp_path / "ck"))
    del a
    b = Tracker(cfg, weights=w)
    b.load_checkpoint(path)
    assert b.frame_index == 3
    rest = run(b, clip[4:])
    for k, (r, g, h) in enumerate(zip(ref, first + rest, again), start=1):
        assert r[0] == g[0] == h[0], f"frame {k}: estimate"
        assert np.array_equal(r[1], g[1]) and np.array_equal(r[1], h[1]), f"frame {k}: ancestors"
        assert np.array_equal(r[2].view(np.uint32), g[2].view(np.uint32)), f"frame {k}: particles"
        assert np.array_equal(r[2].view(np.uint32), h[2].view(np.uint32)), f"frame {k}: particles (rerun)"
    with pytest.raises(ValueError, match="configuration"):
        other = Tracker(load_config({"model": {"arch": "vit_tiny_patch16_224", "dtype": "bf16"},
                                     "particles": {"num": 128, "seed": 99}}), weights=w)
        other.load_checkpoint(path)
    # any value the arithmetic depends on must match, not only P / seed / arch
    for change, key in (({"likelihood": {"lambda": 10.0, "template_update": alpha}}, "lambda"),
                        ({"model": {"dtype": "fp32"}, "likelihood": {"template_update": alpha}}, "dtype"),
                        ({"particles": {"motion_std": [2.0, 2.0, 0.01]}, "likelihood": {"template_update": alpha}},
                         "motion_std")):
        c2 = {"model": {"arch": "vit_tiny_patch16_224", "dtype": "bf16", "weights": {"seed": 3}},
              "particles": {"num": 256, "seed": 99}}
        for sect, vals in change.items():
            c2.setdefault(sect, {}).update(vals)
        with pytest.raises(ValueError, match=key):
            Tracker(load_config(c2), weights=w).load_checkpoint(path)
    # explicit weights of another set (same seed in the config) are refused too
    w2 = make_vit_weights(ARCHS["vit_tiny_patch16_224"], seed=4)
    with pytest.raises(ValueError, match="weights_crc32"):
        Tracker(cfg, weights=w2).load_checkpoint(path)


def test_main_checkpoint_resume(tmp_path):
    """main.py --checkpoint after 3 frames, then --resume for the rest: the positions equal one uninterrupted run."""
    import json
    import sys
    import yaml
    sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
    import main as vpf_main
    cfg = {"model": {"arch": "vit_tiny_patch16_224", "dtype": "bf16"}, "particles": {"num": 128, "seed": 5},
           "input": {"source": "synthetic", "frames": 7}}
    cpath = tmp_path / "config.yaml"
    cpath.write_text(yaml.safe_dump(cfg))
    full, part1, part2 = tmp_path / "full.json", tmp_path / "p1.json", tmp_path / "p2.json"
    ck = str(tmp_path / "state")
    assert vpf_main.main(["--config", str(cpath), "--out", str(full)]) == 0
    assert vpf_main.main(["--config", str(cpath), "--frames", "4", "--out", str(part1), "--checkpoint", ck]) == 0
    assert vpf_main.main(["--config", str(cpath), "--out", str(part2), "--resume", ck]) == 0
    a, b, c = (json.loads(p.read_text()) for p in (full, part1, part2))
    assert [r["frame"] for r in b] == [1, 2, 3] and [r["frame"] for r in c] == [4, 5, 6]
    assert a == b + c
