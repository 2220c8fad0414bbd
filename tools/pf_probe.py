"""Time the device-resident estimate + resample (vpf_estimate_resample: k_stats_scan_global, one 1024-thread
workgroup over all P weights, then k_resample_global, one thread per slot) at the BASELINE configs' particle counts,
for one shard (world 1) and for G gathered shard chunks read through the kernel's strides (the layout every rank
reads at world G). Every rank runs it over the global set each frame, so its cost does not shrink with G
(VERDICT r2 #6). HIP-event averages over `--reps` launches after a warm-up.

    python tools/pf_probe.py [--reps 200]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    import torch

    from vitparticlefiltertracker_amd import ops  # noqa: F401
    from vitparticlefiltertracker_amd.particle_filter import chunk_words, global_view, shard_views
    vpf = torch.ops.vpf
    dev = torch.device("cuda", 0)
    rows = []
    for P in (4096, 16384, 65536):
        for G in (1, 8):
            n = P // G
            g = torch.Generator(device="cpu").manual_seed(P + G)
            allc = torch.zeros(G * chunk_words(n), dtype=torch.int32)
            for r in range(G):
                c = allc[r * chunk_words(n):(r + 1) * chunk_words(n)]
                Q, parts = shard_views(c, n)
                Q.copy_(torch.randint(0, 1 << 40, (n,), generator=g, dtype=torch.int64))
                parts.copy_(torch.rand(3, n, generator=g) * 200)
            allc = allc.to(dev)
            if G == 1:
                Q, parts = shard_views(allc, n)
                view = (Q, n, parts.reshape(-1), n, 3 * n, n)
            else:
                view = global_view(allc, G, n)
            n_out = n                                        # a rank's slots
            anc = torch.empty(n_out, dtype=torch.int32, device=dev)
            states = torch.empty(3, n_out, dtype=torch.float32, device=dev)
            cdf = torch.empty(P, dtype=torch.int64, device=dev)
            stats = torch.empty(4, dtype=torch.int64, device=dev)
            Qv, qs, Pv, ld, ps, nsh = view

            def run():
                vpf.estimate_resample(Qv, qs, Pv, ld, ps, nsh, P, 1234, 7, 0, n_out, anc, states, cdf, stats)
            for _ in range(10):
                run()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.reps):
                run()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) * 1e3 / args.reps
            rows.append({"particles": P, "shards": G, "slots": n_out, "us_per_call": round(us, 2)})
            print(json.dumps(rows[-1]), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
