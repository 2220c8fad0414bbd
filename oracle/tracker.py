"""ORACLE (test infrastructure only): CPU mirror of vitparticlefiltertracker_amd.Tracker (SPEC S8).

Same API shape (init / track / run) so the parity tests read like tests of the product. Every step is a
restatement: predict / crop / estimate / resample from oracle/pf_oracle.c, the ViT from oracle/vit.py
(torch fp32 on CPU). The reference itself has no runnable tracker (README.md:34-42 describe main.py,
which is absent).

`track(frame, Q=None)`: when `Q` is given (e.g. the GPU's int64 weights of the same frame) the oracle's own
likelihood is bypassed — the "feature injection" mode that makes resample parity bit-exact.
"""
from __future__ import annotations

from typing import Optional, Tuple

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
        return est
