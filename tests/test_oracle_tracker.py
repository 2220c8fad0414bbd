"""CPU: the oracle's SPEC S9 pieces (template update, multiple targets) — the checker the §8f-4 GPU tests compare
against. ViT-Ti on a handful of particles (fp32 torch on the CPU, seconds)."""
import copy

import numpy as np

from oracle.tracker import OracleMultiTracker, OracleTracker
from vitparticlefiltertracker_amd.config import ARCHS, load_config
from vitparticlefiltertracker_amd.frames import synthetic_clip
from vitparticlefiltertracker_amd.weights import make_vit_weights

ARCH = ARCHS["vit_tiny_patch16_224"]


def _cfg(alpha, P=8, seed=99):
    return load_config({"model": {"arch": ARCH.name, "dtype": "fp32", "weights": {"seed": 3}},
                        "particles": {"num": P, "seed": seed}, "likelihood": {"template_update": alpha}})


def test_template_update_alpha0_is_identity_and_alpha_blends():
    w = make_vit_weights(ARCH, seed=3)
    clip = synthetic_clip(3)
    fixed, upd = OracleTracker(_cfg(0.0), w, ARCH), OracleTracker(_cfg(0.5), w, ARCH)
    for o in (fixed, upd):
        o.init(clip[0], (80, 80, 64, 64))
    t0 = fixed.template.copy()
    for f in clip[1:]:
        t_before = upd.template.copy()
        fixed.track(f)
        e_upd = upd.track(f)
        assert np.array_equal(fixed.template, t0)                    # alpha = 0: bit-identical template
        # S9 by hand: the feature at the estimate, blended 50/50 with the previous template, renormalised
        fe = upd.features(f, np.array([[e_upd[0]], [e_upd[1]], [e_upd[2]]], np.float32))[0]
        g = 0.5 * t_before + 0.5 * fe / np.linalg.norm(fe)
        np.testing.assert_allclose(upd.template, g / np.linalg.norm(g), rtol=1e-6, atol=1e-7)
        assert abs(np.linalg.norm(upd.template) - 1.0) < 1e-6


def test_multitracker_targets_are_independent_single_trackers():
    """SPEC S9: target k of OracleMultiTracker is exactly an OracleTracker with seed + k on its own box."""
    w = make_vit_weights(ARCH, seed=3)
    clip = synthetic_clip(3)
    boxes = [(70, 70, 48, 48), (100, 90, 64, 40)]
    cfg = _cfg(0.5, P=8, seed=7)
    om = OracleMultiTracker(cfg, 2, w, ARCH)
    om.init(clip[0], boxes)
    singles = []
    for k, b in enumerate(boxes):
        c = copy.deepcopy(cfg)
        c["particles"]["seed"] = 7 + k
        o = OracleTracker(c, w, ARCH)
        o.init(clip[0], b)
        singles.append(o)
    assert om.targets[1].box_wh == (64.0, 40.0)
    for f in clip[1:]:
        ests = om.track(f)
        for k, o in enumerate(singles):
            assert ests[k] == o.track(f)
            assert np.array_equal(om.targets[k].particles, o.particles)
            assert np.array_equal(om.targets[k].template, o.template)
    # the two targets really differ (own seed, own box)
    assert not np.array_equal(om.targets[0].particles, om.targets[1].particles)
