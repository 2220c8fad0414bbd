"""Per-frame host-gap probe: full Tracker.track() loop vs the same frame's device work enqueued back to back
(no host wait per frame) vs the HIP-graph replay alone. python tools/gap_probe.py <particles> [frames]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from vitparticlefiltertracker_amd import Tracker, load_config  # noqa: E402
from vitparticlefiltertracker_amd.frames import synthetic_clip  # noqa: E402

P = int(sys.argv[1])
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
cfg = load_config({"model": {"arch": "vit_base_patch16_224", "dtype": "bf16"}, "particles": {"num": P}})
frames = [torch.from_numpy(f).cuda() for f in synthetic_clip(4 + 3 * K)]
tr = Tracker(cfg)
tr.init(frames[0], cfg["input"]["bbox0"])
for k in range(3):
    tr.track(frames[1 + k])
base = 4


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / K, t_enq * 1e3 / K


def full():
    for k in range(K):
        tr.track(frames[base + k])


def nowait():
    for k in range(K):
        tr._upload(frames[base + K + k])
        tr.frame_index += 1
        tr.pf.predict(tr.frame_index)
        tr.weigh()
        tr.pf._settle()
        tr.pf._commit()


def graph_only():
    for k in range(K):
        tr._graph.replay()


for name, fn in (("track", full), ("no_host_wait", nowait), ("graph_only", graph_only)):
    ms, enq = timed(fn)
    print(f"P={P} {name}: {ms:.3f} ms/frame (host enqueue {enq:.3f} ms/frame)", flush=True)
