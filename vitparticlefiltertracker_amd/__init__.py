"""MI355X-native ViT + particle-filter tracker (drop-in for the hot path of
tugitbartlomiej/ViTParticleFilterTracker; see SPEC.md).

Public API (the names the reference's main.py would use):
  Tracker(cfg).init(frame, bbox); Tracker.track(frame) -> (x, y, scale)
  MultiTracker(cfg, n_objects).init(frame, bboxes); .track(frame) -> [(x, y, scale)] (one batched ViT pass)
  ParticleFilter(...).predict() / .update(features, template) / .estimate() / .resample()
  load_config(path | dict | None)
The compute runs in libvpf.so (hand-written gfx950 HIP kernels) through torch.ops.vpf.* custom ops; there
is no CPU fallback.
"""
from .config import ARCHS, ViTArch, load_config  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # GPU-facing classes import torch / libvpf lazily so `import vitparticlefiltertracker_amd` stays cheap.
    if name == "Tracker":
        from .tracker import Tracker
        return Tracker
    if name == "MultiTracker":
        from .tracker import MultiTracker
        return MultiTracker
    if name == "ParticleFilter":
        from .particle_filter import ParticleFilter
        return ParticleFilter
    if name == "ViTEngine":
        from .vit import ViTEngine
        return ViTEngine
    raise AttributeError(name)
