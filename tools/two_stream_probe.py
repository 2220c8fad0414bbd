"""Probe: does splitting a per-GPU particle batch into two halves on two forked streams (one HIP graph) fill
the GEMM tail waves? Times graph replays of (a) one ViTEngine over n particles, (b) two engines over n/2 each,
captured on two streams forked from the capture stream. Usage: python tools/two_stream_probe.py [n ...]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitparticlefiltertracker_amd.config import ARCHS  # noqa: E402
from vitparticlefiltertracker_amd.vit import ViTEngine  # noqa: E402
from vitparticlefiltertracker_amd.weights import make_vit_weights  # noqa: E402


def timed(g, reps=10):
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    dev = torch.device("cuda:0")
    arch = ARCHS["vit_base_patch16_224"]
    w = make_vit_weights(arch, seed=0)
    frame = torch.randint(0, 256, (224, 224, 3), dtype=torch.uint8, device=dev)
    tmpl = torch.nn.functional.normalize(torch.randn(arch.dim, device=dev), dim=0)
    for n in [int(a) for a in sys.argv[1:]] or [512, 1024, 4096]:
        parts = torch.empty(3, n, device=dev)
        parts[0].uniform_(90, 130)
        parts[1].uniform_(90, 130)
        parts[2].uniform_(0.9, 1.1)
        e1 = ViTEngine(arch, w, "bf16", dev, n)
        K = int(os.environ.get("PROBE_SPLITS", "2"))
        cuts = [n * i // K for i in range(K + 1)]
        halves = [ViTEngine(arch, w, "bf16", dev, cuts[i + 1] - cuts[i]) for i in range(K)]
        ph = [parts[:, cuts[i]:cuts[i + 1]].contiguous() for i in range(K)]
        box = (64.0, 64.0)

        def one():
            e1.forward_weights(frame, parts, box, tmpl, 8.0, 40)

        streams = [torch.cuda.Stream(device=dev) for _ in range(K)]

        def two():
            cur = torch.cuda.current_stream()
            for s, e, p in zip(streams, halves, ph):
                s.wait_stream(cur)
                with torch.cuda.stream(s):
                    e.forward_weights(frame, p, box, tmpl, 8.0, 40)
            for s in streams:
                cur.wait_stream(s)

        res = {}
        for name, fn in (("one", one), ("two", two)):
            fn()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                fn()
            res[name] = timed(g)
        q1 = e1.Q[:n].cpu()
        q2 = torch.cat([e.Q[: cuts[i + 1] - cuts[i]] for i, e in enumerate(halves)]).cpu()
        print(f"n={n} splits={K}: one {res['one']:.3f} ms  split {res['two']:.3f} ms  ratio {res['two'] / res['one']:.4f}"
              f"  Q equal: {bool(torch.equal(q1, q2))}", flush=True)
        del e1, halves
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
