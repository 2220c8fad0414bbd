"""ORACLE (test infrastructure only): CPU mirror of vitparticlefiltertracker_amd.Tracker (SPEC S8).

Same API shape (init / track / run) so the parity tests read like tests of the product. Every step is a
restatement: predict / crop / estimate / resample from oracle/pf_oracle.c, the ViT from oracle/vit.py
(torch fp32 on CPU). The reference itself has no runnable tracker (README.md:34-42 describe main.py,
which is absent).

`track(frame, Q=None)`: when `Q` is given (e.g. the GPU's int64 weights of the same frame) the oracle's own
likelihood is bypassed — the "feature injection" mode that makes resample parity bit-exact.

SPEC S9 (§8f rank 4): `likelihood.template_update` = alpha updates the template after each frame's estimate from the
feature at that estimate (`OracleTracker.update_template`); `OracleMultiTracker` runs K targets, each with its own box,
template and particle seed (seed + k), as independent single-target trackers.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import pf
from . import vit as ovit


class OracleTracker:
    def __init__(self, cfg: dict, weights, arch, threads: Optional[int] = None):
        self.cfg, self.w, self.arch = cfg, weights, arch
        if threads:
            torch.set_num_threads(int(threads))
        p = cfg["particles"]
        self.P = int(p["num"])
        self.motion_std = [float(v) for v in p["motion_std"]]
        self.scale_range = [float(v) for v in p["scale_range"]]
        self.seed = int(p["seed"])
        self.lam = float(cfg["likelihood"]["lambda"])
        self.bits = int(cfg["likelihood"]["weight_bits"])
        self.mean, self.std = cfg["model"]["mean"], cfg["model"]["std"]
        self.alpha = float(cfg["likelihood"].get("template_update", 0.0))
        self.particles = None
        self.template = None
        self.frame_index = 0
        self.last_Q = None
        self.last_ancestors = None

    def features(self, frame: np.ndarray, particles: np.ndarray, chunk: int = 64) -> np.ndarray:
        A = self.arch
        out = []
        for i in range(0, particles.shape[1], chunk):
            sub = np.ascontiguousarray(particles[:, i:i + chunk])
            patches = pf.crop_patches(frame, sub, self.box_wh, A.img_size, A.patch, A.patch_kp, self.mean, self.std)
            out.append(ovit.features_from_patches(torch.from_numpy(patches), self.w, A).numpy())
        return np.concatenate(out, 0)

    def init(self, frame: np.ndarray, bbox) -> None:
        bx, by, bw, bh = (float(v) for v in bbox)
        self.box_wh = (bw, bh)
        cx, cy = bx + 0.5 * bw, by + 0.5 * bh
        one = np.array([[cx], [cy], [1.0]], np.float32)
        f = self.features(frame, one)[0].astype(np.float32)
        self.template = (f / np.linalg.norm(f)).astype(np.float32)
        self.particles = np.empty((3, self.P), np.float32)
        self.particles[0], self.particles[1], self.particles[2] = np.float32(cx), np.float32(cy), np.float32(1.0)
        self.H, self.W = frame.shape[0], frame.shape[1]
        self.frame_index = 0

    def likelihood(self, feats: np.ndarray) -> np.ndarray:
        f = feats.astype(np.float32)
        nrm = np.linalg.norm(f, axis=1)
        with np.errstate(invalid="ignore", divide="ignore"):
            sim = np.where(nrm > 0, (f @ self.template) / np.where(nrm > 0, nrm, 1), 0)   # zero row: sim 0
        sim[~np.isfinite(nrm)] = np.nan                                          # SPEC S5: non-finite -> Q 0
        return pf.weights_to_Q(sim.astype(np.float32), self.lam, self.bits)

    def track(self, frame: np.ndarray, Q: Optional[np.ndarray] = None) -> Tuple[float, float, float]:
        self.frame_index += 1
        pf.predict(self.particles, 0, self.seed, self.frame_index, self.motion_std, self.W, self.H, self.scale_range)
        if Q is None:
            Q = self.likelihood(self.features(frame, self.particles))
        Q = np.ascontiguousarray(Q, np.int64)
        self.last_Q = Q
        est = pf.estimate(Q, self.particles)
        Qr = Q if Q.sum() > 0 else np.zeros_like(Q)
        anc = pf.resample(Qr, pf.resample_U(self.seed, self.frame_index))
        self.last_ancestors = anc
        self.particles = np.ascontiguousarray(self.particles[:, anc])
        if self.alpha > 0.0:
            self.update_template(frame, est)
        return est

    def update_template(self, frame: np.ndarray, state, alpha: Optional[float] = None) -> None:
        """SPEC S9: t <- g / |g|, g = (1 - alpha) t + alpha f / |f|, f the feature of the crop at `state` (fp32) with
        the template box on this frame; fp32 arithmetic."""
        a = np.float32(self.alpha if alpha is None else alpha)
        st = np.array([[state[0]], [state[1]], [state[2]]], np.float32)
        f = self.features(frame, st)[0].astype(np.float32)
        g = (np.float32(1.0) - a) * self.template + a * (f / np.linalg.norm(f))
        self.template = (g / np.linalg.norm(g)).astype(np.float32)


class OracleMultiTracker:
    """SPEC S9 multi-object mirror of vitparticlefiltertracker_amd.MultiTracker: target k is an OracleTracker with the
    particle seed particles.seed + k, initialised on its own box (so it crops with its own template box and weighs
    against its own template), and template-updated from its own estimate when likelihood.template_update > 0."""

    def __init__(self, cfg: dict, n_objects: int, weights, arch, threads: Optional[int] = None):
        import copy
        self.K = int(n_objects)
        self.targets: List[OracleTracker] = []
        for k in range(self.K):
            c = copy.deepcopy(cfg)
            c["particles"]["seed"] = int(cfg["particles"]["seed"]) + k
            self.targets.append(OracleTracker(c, weights, arch, threads if k == 0 else None))

    def init(self, frame: np.ndarray, bboxes: Sequence) -> None:
        if len(bboxes) != self.K:
            raise ValueError(f"expected {self.K} boxes")
        for t, b in zip(self.targets, bboxes):
            t.init(frame, b)

    def track(self, frame: np.ndarray, Qs: Optional[Sequence[np.ndarray]] = None) -> List[Tuple[float, float, float]]:
        """One frame for every target; `Qs[k]` (optional) injects target k's weights as OracleTracker.track does."""
        return [t.track(frame, None if Qs is None else Qs[k]) for k, t in enumerate(self.targets)]
