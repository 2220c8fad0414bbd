"""`Tracker` — the per-frame loop the reference drives from main.py ("integrates the Vision Transformer
(ViT) architecture with a Particle Filter to achieve precise object position tracking",
/root/reference/README.md:3; "provide the input data ... configure ... config.yaml ... output the tracked
positions", README.md:42). SPEC.md S8 / SURVEY.md §8a H13-H14.

    t = Tracker("config.yaml")        # or a dict, or None for the defaults
    t.init(frame0, (x, y, w, h))      # template feature from the bbox crop (H13)
    for f in frames: x, y, s = t.track(f)

Per frame: predict (eager launch; its frame index is a kernel argument) -> [HIP graph replay: crop+ViT
-> final LN -> cosine -> Q] -> (world > 1: one all-gather of the shard chunks) -> estimate + resample on the
device (vpf_estimate_resample). The only host synchronisation is reading the 32-B estimate statistics.
"""
from __future__ import annotations

import os
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from .config import arch_of, load_config
from .particle_filter import ParticleFilter, shard_range
from .vit import ViTEngine
from .weights import make_vit_weights


def weights_digest(weights) -> str:
    """crc32 over every weight tensor's bytes (sorted names, fp32): the configuration fingerprint records it, so a
    checkpoint taken with one weight set is refused by a tracker built with another, whether the weights came from
    the seed or from the `weights=` argument."""
    import zlib
    crc = 0
    for name in sorted(weights):
        t = weights[name].detach().to("cpu", torch.float32).contiguous()
        crc = zlib.crc32(name.encode(), crc)
        crc = zlib.crc32(t.numpy().tobytes(), crc)
    return f"{crc:08x}"


# 3: the fingerprint includes the weights' crc32 (round 4 added it to format 2 without a bump: ADVICE r4)
CHECKPOINT_FORMAT = 3


def _stage_frame(self, frame) -> torch.Tensor:
    """Frame -> the device frame buffer `self._frame_dev` (Tracker and MultiTracker): a device tensor is copied on the
    device; a pinned uint8[H][W][3] tensor (frames.prefetch) is copied asynchronously; anything else goes through a
    pinned staging buffer `self._frame_host` and an asynchronous copy guarded by the event `self._h2d_done`, so the host
    never blocks on the H2D copy of the frame it just submitted. A new frame shape drops the captured graph."""
    if isinstance(frame, torch.Tensor) and frame.is_cuda:
        src = frame.to(torch.uint8)
        if self._frame_dev is None or self._frame_dev.shape != src.shape:
            self._frame_dev = torch.empty_like(src)
            self._graph = None
        self._frame_dev.copy_(src)
        return self._frame_dev
    if (isinstance(frame, torch.Tensor) and frame.dtype == torch.uint8 and frame.dim() == 3
            and frame.shape[2] == 3 and frame.is_contiguous() and frame.is_pinned()):
        # frames.prefetch() output: already staged in pinned memory, copy straight from it
        if self._frame_dev is None or self._frame_dev.shape != frame.shape:
            self._frame_dev = torch.empty(frame.shape, dtype=torch.uint8, device=self.device)
            self._graph = None
        self._frame_dev.copy_(frame, non_blocking=True)
        return self._frame_dev
    arr = np.ascontiguousarray(frame.cpu().numpy() if isinstance(frame, torch.Tensor) else frame, dtype=np.uint8)
    if arr.ndim != 3 or arr.shape[2] != 3:
        raise ValueError("frame must be uint8[H][W][3]")
    if self._frame_dev is None or tuple(self._frame_dev.shape) != arr.shape:
        self._frame_dev = torch.empty(arr.shape, dtype=torch.uint8, device=self.device)
        self._graph = None
    # the pinned staging buffer is sized independently: the device frame may have come from a pinned or
    # device tensor of this shape, which never touches it
    if self._frame_host is None or tuple(self._frame_host.shape) != arr.shape:
        # the previous async copy may still read the old buffer: finish it before dropping it
        if self._frame_host is not None:
            torch.cuda.current_stream(self.device).synchronize()
        self._frame_host = torch.empty(arr.shape, dtype=torch.uint8).pin_memory()
    elif self._h2d_done is not None:
        # reusing the staging buffer: the last frame's H2D copy must have finished reading it
        self._h2d_done.synchronize()
    self._frame_host.numpy()[...] = arr
    self._frame_dev.copy_(self._frame_host, non_blocking=True)
    if self._h2d_done is None:
        self._h2d_done = torch.cuda.Event()
    self._h2d_done.record()
    return self._frame_dev


class _LazyDigest:
    """`weights_digest` of the tracker's weights. Weights built from the seed: computed on first use (a checkpoint save /
    load) from a rebuild (make_vit_weights is deterministic) and cached, since the crc32 converts every weight to a host
    fp32 copy (~1.2 GB for ViT-L/14) that a tracker which never checkpoints should not pay. Weights passed
    in: digested at construction (`_set_weights_digest`) and not referenced afterwards, so the caller can free them and
    a later change to the caller's tensors cannot make the recorded crc describe other weights than the engine's copy
    (ADVICE r5)."""

    def _set_weights_digest(self, weights) -> None:
        self._digest = weights_digest(weights) if weights is not None else None

    @property
    def weights_digest(self) -> str:
        if self._digest is None:
            self._digest = weights_digest(make_vit_weights(self.arch, seed=int(self.cfg["model"]["weights"]["seed"])))
        return self._digest


def _fingerprint(cfg, arch_name: str, digest: str, rank: int, world_size: int) -> dict:
    """Every configuration value a tracking frame's arithmetic depends on: a checkpoint records these and
    a resume under any other value is refused instead of drifting from the original run."""
    m, p, lk = cfg["model"], cfg["particles"], cfg["likelihood"]
    return {"arch": arch_name, "dtype": str(m["dtype"]), "weights_seed": int(m["weights"]["seed"]),
            "weights_crc32": digest,
            "mean": [float(v) for v in m["mean"]], "std": [float(v) for v in m["std"]],
            "P": int(p["num"]), "motion_std": [float(v) for v in p["motion_std"]],
            "scale_range": [float(v) for v in p["scale_range"]], "seed": int(p["seed"]),
            "lambda": float(lk["lambda"]), "weight_bits": int(lk["weight_bits"]),
            "template_update": float(lk["template_update"]), "rank": rank, "world_size": world_size}


def _check_fingerprint(sd: dict, mine: dict) -> None:
    import json
    fmt = int(sd["format"])
    if fmt == 1:
        raise ValueError("checkpoint format 1 (rounds 1-2) records only P, rank, world size, seed and arch; format "
                         f"{CHECKPOINT_FORMAT} also checks every value the tracking arithmetic depends on (dtype, lambda, "
                         "motion, weights, ...): re-create the checkpoint with this version")
    if fmt not in (2, CHECKPOINT_FORMAT):
        raise ValueError(f"unknown checkpoint format {fmt}")
    saved = json.loads(str(sd["config"]))
    # format 2 is format 3 without the bump (round 4 added the crc to format 2's fingerprint): such a file carries the
    # crc and is checked like format 3; a format-2 file written before that lacks it and is refused
    if fmt == 2 and "weights_crc32" not in saved:
        raise ValueError("this format-2 checkpoint predates the weights' crc32 in the fingerprint, which format "
                         f"{CHECKPOINT_FORMAT} checks so that a resume with other weights is refused: re-create the "
                         "checkpoint with this version")
    diff = sorted(k for k in set(saved) | set(mine) if saved.get(k) != mine.get(k))
    if diff:
        raise ValueError("checkpoint was written by a tracker with another configuration or rank layout: "
                         + ", ".join(f"{k} {saved.get(k)!r} != {mine.get(k)!r}" for k in diff))


def _sd_particles_soa(sd: dict) -> np.ndarray:
    """A checkpoint's particle states in the SoA layout (float32[3][P_l], [K][3][P_l] for a MultiTracker). Since round 6
    the key is `particles_soa`: `ParticleFilter.particles` became the [P_l][3] view in round 5, and one name for two
    shapes invited misreads. Files of earlier rounds store the same SoA array under `particles`."""
    a = sd["particles_soa"] if "particles_soa" in sd else sd["particles"]
    return np.ascontiguousarray(a, dtype=np.float32)


def _checkpoint_file(path: str, rank: int, world_size: int) -> str:
    """`<path>.rank<r>of<G>.npz` with several ranks, `<path>.npz` with one; a path that already names this rank's
    file (what save_checkpoint returned) is taken as is, so save -> load round-trips either way."""
    suffix = f".rank{rank}of{world_size}.npz" if world_size > 1 else ".npz"
    return path if path.endswith(suffix) else path + suffix


def _blend_template(t: torch.Tensor, f: torch.Tensor, alpha: float) -> None:
    """SPEC S9 in place on the device: t <- g / |g|, g = (1 - alpha) t + alpha f / |f| (fp32)."""
    g = (1.0 - alpha) * t + alpha * (f / f.norm())
    t.copy_(g / g.norm())


def _dist_info(rank, world_size, group):
    if rank is not None and world_size is not None:
        return int(rank), int(world_size), group
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group), group
    return 0, 1, None


class Tracker(_LazyDigest):
    def __init__(self, cfg=None, device=None, rank: Optional[int] = None, world_size: Optional[int] = None,
                 group=None, use_graph: bool = True, weights=None):
        self.cfg = load_config(cfg)
        if not torch.cuda.is_available():
            raise _lib.VPFError("Tracker runs on the HIP device only; the CPU restatement is oracle/ (tests)")
        self.rank, self.world_size, self.group = _dist_info(rank, world_size, group)
        if device is None:
            local = int(os.environ.get("LOCAL_RANK", self.rank % max(1, torch.cuda.device_count())))
            device = torch.device("cuda", local)
        self.device = torch.device(device)
        torch.cuda.set_device(self.device)
        c = self.cfg
        self.arch = arch_of(c)
        P = int(c["particles"]["num"])
        _, self.n_local = shard_range(P, self.world_size, self.rank)   # rank r: [floor(rP/G), floor((r+1)P/G))
        w = weights if weights is not None else make_vit_weights(self.arch, seed=int(c["model"]["weights"]["seed"]))
        self._set_weights_digest(weights)
        self.engine = ViTEngine(self.arch, w, c["model"]["dtype"], self.device, max(1, self.n_local),
                                c["model"]["mean"], c["model"]["std"])
        self.lam = float(c["likelihood"]["lambda"])
        self.bits = int(c["likelihood"]["weight_bits"])
        self.template_alpha = float(c["likelihood"]["template_update"])
        self.use_graph = bool(use_graph)
        self.pf: Optional[ParticleFilter] = None
        self.template: Optional[torch.Tensor] = None
        self.box_wh: Optional[Tuple[float, float]] = None
        self._frame_dev: Optional[torch.Tensor] = None
        self._frame_host: Optional[torch.Tensor] = None
        self._h2d_done: Optional[torch.cuda.Event] = None
        self._graph: Optional[torch.cuda.CUDAGraph] = None
        self.frame_index = 0

    # ------------------------------------------------------------------ frames
    def _upload(self, frame) -> torch.Tensor:
        return _stage_frame(self, frame)

    # ------------------------------------------------------------------ H13
    def init(self, frame, bbox) -> None:
        """Template from the bbox (x, y, w, h) crop at scale 1; particles reset to the bbox centre."""
        fd = self._upload(frame)
        bx, by, bw, bh = (float(v) for v in bbox)
        self.box_wh = (bw, bh)
        cx, cy = bx + 0.5 * bw, by + 0.5 * bh
        one = torch.tensor([[cx], [cy], [1.0]], dtype=torch.float32, device=self.device)
        f = self.engine.features(fd, one, self.box_wh)[0].clone()
        self.template = (f / f.norm()).contiguous()
        c = self.cfg
        if self.pf is None:
            self.pf = ParticleFilter(int(c["particles"]["num"]), (cx, cy, 1.0), c["particles"]["motion_std"],
                                     c["particles"]["scale_range"], int(c["particles"]["seed"]), self.device,
                                     (fd.shape[0], fd.shape[1]), self.lam, self.bits, self.rank, self.world_size,
                                     self.group)
        else:
            self.pf.height, self.pf.width = fd.shape[0], fd.shape[1]
            self.pf.reset((cx, cy, 1.0))
        self._graph = None
        self.frame_index = 0

    # ------------------------------------------------------------------ H14
    def _features_to_weights(self) -> None:
        self.engine.forward_weights(self._frame_dev, self.pf.particles_soa, self.box_wh, self.template, self.lam,
                                    self.bits)

    def _capture(self) -> None:
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self._features_to_weights()   # warm-up outside capture
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        # thread_local: RCCL's watchdog thread queries events while a capture runs (multi-GPU); "global" would
        # invalidate the capture on that, the capture itself only involves this thread's stream
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            self._features_to_weights()
        self._graph = g

    def weigh(self) -> None:
        """Crop + ViT + weights for the current particles and uploaded frame (graph replay when enabled)."""
        if self.use_graph:
            if self._graph is None:
                self._capture()
            self._graph.replay()
        else:
            self._features_to_weights()
        self.pf.set_weights(self.engine.Q[: self.n_local])

    def track(self, frame) -> Tuple[float, float, float]:
        if self.pf is None:
            raise RuntimeError("call init(frame, bbox) first")
        fd = self._upload(frame)
        if (fd.shape[0], fd.shape[1]) != (self.pf.height, self.pf.width):
            # a frame of another size: predict clamps to the new bounds (the graph was dropped by _upload)
            self.pf.height, self.pf.width = int(fd.shape[0]), int(fd.shape[1])
        self.frame_index += 1
        self.pf.predict(self.frame_index)
        self.weigh()
        # estimate + resample on the device, the resample enqueued before the host reads the estimate; the template
        # update crops at the estimate on this frame and does not read the particles
        est = self.pf.step()
        if self.template_alpha > 0.0:
            self.update_template(est)
        return est

    def update_template(self, state, alpha: Optional[float] = None) -> None:
        """Template update (SPEC S9): t <- normalise((1 - alpha) t + alpha f / |f|) with f the
        CLS feature of the crop at `state` = (x, y, scale) of the current frame. In place, so the captured graph
        keeps reading the same buffer; every rank computes the same bits (same estimate, same kernels)."""
        a = self.template_alpha if alpha is None else float(alpha)
        st = torch.tensor([[state[0]], [state[1]], [state[2]]], dtype=torch.float32, device=self.device)
        f = self.engine.features(self._frame_dev, st, self.box_wh)[0]
        _blend_template(self.template, f, a)

    # ------------------------------------------------------------------ checkpoint / resume
    def config_fingerprint(self) -> dict:
        """Every configuration value a tracking frame's arithmetic depends on: a checkpoint records
        these and a resume under any other value is refused instead of drifting from the original run."""
        return _fingerprint(self.cfg, self.arch.name, self.weights_digest, self.rank, self.world_size)

    def state_dict(self) -> dict:
        """The tracker's state between frames as numpy arrays: this rank's particles as `particles_soa` (float32[3][P_l],
        the SoA storage; `ParticleFilter.particles` is its [P_l][3] view) after the last resample (so Q is zero), the
        template, the template box, the frame size and the frame index, plus the configuration
        fingerprint (JSON). The motion noise and the resample word are counter-based (seed, frame index, global
        particle index: SPEC S1/S2), so a tracker with the same configuration that loads this continues bit for
        bit."""
        import json
        if self.pf is None:
            raise RuntimeError("call init(frame, bbox) first")
        return {"format": np.int64(CHECKPOINT_FORMAT), "frame_index": np.int64(self.frame_index),
                "pf_frame": np.int64(self.pf.frame), "particles_soa": self.pf.particles_soa.cpu().numpy(),
                "template": self.template.cpu().numpy(), "box_wh": np.array(self.box_wh, np.float64),
                "frame_hw": np.array([self.pf.height, self.pf.width], np.int64),
                "config": np.array(json.dumps(self.config_fingerprint(), sort_keys=True))}

    def load_state_dict(self, sd: dict) -> None:
        _check_fingerprint(sd, self.config_fingerprint())
        if "n_objects" in sd:
            raise ValueError("this checkpoint was written by a MultiTracker")
        c = self.cfg
        H, W = (int(v) for v in sd["frame_hw"])
        self.box_wh = tuple(float(v) for v in sd["box_wh"])
        t = torch.from_numpy(np.ascontiguousarray(sd["template"], dtype=np.float32)).to(self.device)
        if self.template is None or self.template.shape != t.shape:
            self.template = t.contiguous()
        else:
            self.template.copy_(t)          # in place: a captured graph reads this buffer
        if self.pf is None:
            self.pf = ParticleFilter(int(c["particles"]["num"]), (0.0, 0.0, 1.0), c["particles"]["motion_std"],
                                     c["particles"]["scale_range"], int(c["particles"]["seed"]), self.device, (H, W),
                                     self.lam, self.bits, self.rank, self.world_size, self.group)
        self.pf.reset((0.0, 0.0, 1.0))
        self.pf.height, self.pf.width = H, W
        self.pf.particles_soa.copy_(torch.from_numpy(_sd_particles_soa(sd)))
        self.pf.frame = int(sd["pf_frame"])
        self.frame_index = int(sd["frame_index"])
        self._graph = None

    def _checkpoint_file(self, path: str) -> str:
        return _checkpoint_file(path, self.rank, self.world_size)

    def save_checkpoint(self, path: str) -> str:
        """np.savez of state_dict() (no pickled objects); with several ranks each writes `<path>.rank<r>of<G>.npz`.
        Returns the file written (load_checkpoint accepts it, or the base path)."""
        path = self._checkpoint_file(path)
        np.savez(path, **self.state_dict())
        return path

    def load_checkpoint(self, path: str) -> None:
        path = self._checkpoint_file(path)
        with np.load(path, allow_pickle=False) as z:
            self.load_state_dict({k: z[k] for k in z.files})

    def box(self, state) -> Tuple[float, float, float, float]:
        """(x, y, w, h) of the box a state (centre x, y, scale) stands for (SPEC S3: scale x template size)."""
        x, y, s = (float(v) for v in state)
        w, h = s * self.box_wh[0], s * self.box_wh[1]
        return x - 0.5 * w, y - 0.5 * h, w, h

    def run(self, frames: Iterable) -> np.ndarray:
        return np.array([self.track(f) for f in frames], dtype=np.float64)


class MultiTracker(_LazyDigest):
    """Several targets in one frame loop (SPEC S9): one ParticleFilter per target, and ONE
    batched ViT forward over every target's particles per frame (crops with each target's own template box, one patch
    GEMM / encoder / final LN over all K*P crops, cosine weights against each target's own template), captured
    into one HIP graph. Target k's particle stream is seeded with particles.seed + k, so a MultiTracker with one
    target reproduces Tracker bit for bit. With likelihood.template_update = alpha > 0 every target's template is
    updated from its own estimate after each frame (one batched feature pass over the K estimate crops).
    Several ranks (as Tracker): every target's particles are sharded by index range over the ranks, each rank runs
    the ViT over its K x P/G crops, and each target's filter does its own chunk all-gather + global estimate /
    resample, so every rank returns the same K estimates, bit-identical to one rank."""

    def __init__(self, cfg=None, n_objects: int = 1, device=None, use_graph: bool = True, weights=None,
                 rank: Optional[int] = None, world_size: Optional[int] = None, group=None):
        self.cfg = load_config(cfg)
        if not torch.cuda.is_available():
            raise _lib.VPFError("MultiTracker runs on the HIP device only")
        if n_objects < 1:
            raise ValueError("n_objects >= 1")
        self.rank, self.world_size, self.group = _dist_info(rank, world_size, group)
        if device is None:
            local = int(os.environ.get("LOCAL_RANK", self.rank % max(1, torch.cuda.device_count())))
            device = torch.device("cuda", local)
        self.device = torch.device(device)
        torch.cuda.set_device(self.device)
        c = self.cfg
        self.arch = arch_of(c)
        self.K = int(n_objects)
        self.P = int(c["particles"]["num"])
        _, self.n_local = shard_range(self.P, self.world_size, self.rank)
        w = weights if weights is not None else make_vit_weights(self.arch, seed=int(c["model"]["weights"]["seed"]))
        self._set_weights_digest(weights)
        self.engine = ViTEngine(self.arch, w, c["model"]["dtype"], self.device, self.K * self.n_local,
                                c["model"]["mean"], c["model"]["std"])
        self.lam = float(c["likelihood"]["lambda"])
        self.bits = int(c["likelihood"]["weight_bits"])
        self.template_alpha = float(c["likelihood"]["template_update"])
        self.use_graph = bool(use_graph)
        self.pfs: List[ParticleFilter] = []
        self.templates: List[torch.Tensor] = []
        self.boxes: List[Tuple[float, float]] = []
        self._frame_dev: Optional[torch.Tensor] = None
        self._frame_host: Optional[torch.Tensor] = None
        self._h2d_done: Optional[torch.cuda.Event] = None
        self._graph = None
        self.frame_index = 0

    def _upload(self, frame) -> torch.Tensor:
        return _stage_frame(self, frame)   # pinned staging + async copy, as Tracker

    def init(self, frame, bboxes: Sequence) -> None:
        if len(bboxes) != self.K:
            raise ValueError(f"expected {self.K} boxes")
        fd = self._upload(frame)
        c = self.cfg
        self.pfs, self.templates, self.boxes = [], [], []
        for k, (bx, by, bw, bh) in enumerate(bboxes):
            bx, by, bw, bh = float(bx), float(by), float(bw), float(bh)
            cx, cy = bx + 0.5 * bw, by + 0.5 * bh
            one = torch.tensor([[cx], [cy], [1.0]], dtype=torch.float32, device=self.device)
            f = self.engine.features(fd, one, (bw, bh))[0].clone()
            self.templates.append((f / f.norm()).contiguous())
            self.boxes.append((bw, bh))
            self.pfs.append(ParticleFilter(self.P, (cx, cy, 1.0), c["particles"]["motion_std"],
                                           c["particles"]["scale_range"], int(c["particles"]["seed"]) + k,
                                           self.device, (fd.shape[0], fd.shape[1]), self.lam, self.bits,
                                           self.rank, self.world_size, self.group))
        self._graph = None
        self.frame_index = 0

    def _forward(self) -> None:
        eng = self.engine
        n = eng.embed_many(self._frame_dev, [pf.particles_soa for pf in self.pfs], self.boxes)
        eng.encoder(n)
        for k in range(self.K):
            eng.weights_from_tokens(self.n_local, self.templates[k], self.lam, self.bits, row0=k * self.n_local)

    def _capture(self) -> None:
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self._forward()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        # thread_local: RCCL's watchdog thread queries events while a capture runs (multi-GPU); "global" would
        # invalidate the capture on that, the capture itself only involves this thread's stream
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            self._forward()
        self._graph = g

    def weigh(self) -> None:
        """Crop + ViT + weights of every target's predicted particles on the uploaded frame (graph replay when
        enabled); each filter's Q is set."""
        if self.use_graph:
            if self._graph is None:
                self._capture()
            self._graph.replay()
        else:
            self._forward()
        for k, pf in enumerate(self.pfs):
            pf.set_weights(self.engine.Q[k * self.n_local:(k + 1) * self.n_local])

    def step(self) -> List[Tuple[float, float, float]]:
        """Every target's estimate + resample (all enqueued, then one wait), then the template updates."""
        for pf in self.pfs:
            pf._settle()
            pf._commit()
        ests = [pf._read_estimate() for pf in self.pfs]
        if self.template_alpha > 0.0:
            self.update_templates(ests)
        return ests

    def update_templates(self, states, alpha: Optional[float] = None) -> None:
        """SPEC S9 for every target: t_k <- normalise((1 - alpha) t_k + alpha f_k / |f_k|), f_k the feature of the crop
        at states[k] with target k's box, all K crops in one batched pass. In place (the graph reads the buffers)."""
        a = self.template_alpha if alpha is None else float(alpha)
        sets = [torch.tensor([[st[0]], [st[1]], [st[2]]], dtype=torch.float32, device=self.device) for st in states]
        f = self.engine.features_many(self._frame_dev, sets, self.boxes)
        for k in range(self.K):
            _blend_template(self.templates[k], f[k], a)

    # ------------------------------------------------------------------ checkpoint / resume (as Tracker)
    def config_fingerprint(self) -> dict:
        return {**_fingerprint(self.cfg, self.arch.name, self.weights_digest, self.rank, self.world_size),
                "n_objects": self.K}

    def state_dict(self) -> dict:
        """Tracker.state_dict for every target: particles_soa [K][3][P_l], templates [K][D], template boxes [K][2],
        each filter's frame counter, the frame size and index, and the fingerprint (with the target count)."""
        import json
        if not self.pfs:
            raise RuntimeError("call init(frame, bboxes) first")
        return {"format": np.int64(CHECKPOINT_FORMAT), "n_objects": np.int64(self.K), "frame_index": np.int64(self.frame_index),
                "pf_frame": np.array([pf.frame for pf in self.pfs], np.int64),
                "particles_soa": np.stack([pf.particles_soa.cpu().numpy() for pf in self.pfs]),
                "template": np.stack([t.cpu().numpy() for t in self.templates]),
                "box_wh": np.array(self.boxes, np.float64),
                "frame_hw": np.array([self.pfs[0].height, self.pfs[0].width], np.int64),
                "config": np.array(json.dumps(self.config_fingerprint(), sort_keys=True))}

    def load_state_dict(self, sd: dict) -> None:
        if "n_objects" not in sd:
            raise ValueError("this checkpoint was written by a single-target Tracker")
        _check_fingerprint(sd, self.config_fingerprint())
        c = self.cfg
        H, W = (int(v) for v in sd["frame_hw"])
        boxes = [tuple(float(v) for v in b) for b in sd["box_wh"]]
        if not self.pfs:
            self.pfs = [ParticleFilter(self.P, (0.0, 0.0, 1.0), c["particles"]["motion_std"],
                                       c["particles"]["scale_range"], int(c["particles"]["seed"]) + k, self.device,
                                       (H, W), self.lam, self.bits, self.rank, self.world_size, self.group)
                        for k in range(self.K)]
            self.templates = [torch.empty(self.arch.dim, dtype=torch.float32, device=self.device)
                              for _ in range(self.K)]
        self.boxes = boxes
        for k, pf in enumerate(self.pfs):
            pf.reset((0.0, 0.0, 1.0))
            pf.height, pf.width = H, W
            pf.particles_soa.copy_(torch.from_numpy(np.ascontiguousarray(_sd_particles_soa(sd)[k])))
            pf.frame = int(sd["pf_frame"][k])
            # in place: a captured graph reads these buffers
            self.templates[k].copy_(torch.from_numpy(np.ascontiguousarray(sd["template"][k], dtype=np.float32)))
        self.frame_index = int(sd["frame_index"])
        self._graph = None

    def save_checkpoint(self, path: str) -> str:
        path = _checkpoint_file(path, self.rank, self.world_size)
        np.savez(path, **self.state_dict())
        return path

    def load_checkpoint(self, path: str) -> None:
        with np.load(_checkpoint_file(path, self.rank, self.world_size), allow_pickle=False) as z:
            self.load_state_dict({k: z[k] for k in z.files})

    def track(self, frame) -> List[Tuple[float, float, float]]:
        if not self.pfs:
            raise RuntimeError("call init(frame, bboxes) first")
        fd = self._upload(frame)
        self.frame_index += 1
        for pf in self.pfs:
            pf.height, pf.width = int(fd.shape[0]), int(fd.shape[1])
            pf.predict(self.frame_index)
        self.weigh()
        return self.step()
