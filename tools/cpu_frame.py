"""Time ONE full tracking frame of the CPU oracle at the metric's workload — 4096 particles, ViT-B/16 fp32 (torch
CPU) + the C particle-filter ops (oracle/tracker.py OracleTracker.track) — next to bench.py's bounded-sample
cpu_baseline in the same process, so the extrapolation bench.py reports is checked against a measured frame
(VERDICT r2 #3). Test / measurement infrastructure: the oracle is the checker and the CPU baseline, never the product.

    python tools/cpu_frame.py [--particles 4096] [--arch vit_base_patch16_224] [--threads 0] [--sample-seconds 15]

Progress goes to stderr every 256 crops; one JSON line to stdout.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--particles", type=int, default=4096)
    ap.add_argument("--arch", default="vit_base_patch16_224")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--sample-seconds", type=float, default=15.0)
    ap.add_argument("--batch", type=int, default=8, help="crops per oracle ViT call (bench.py cpu_baseline: 8)")
    args = ap.parse_args()

    import numpy as np
    import torch

    import bench
    from oracle.tracker import OracleTracker
    from vitparticlefiltertracker_amd.config import ARCHS, load_config
    from vitparticlefiltertracker_amd.frames import synthetic_clip
    from vitparticlefiltertracker_amd.weights import make_vit_weights

    cpus = bench.host_cpus()
    threads = args.threads or cpus["threads"]
    torch.set_num_threads(threads)
    arch = ARCHS[args.arch]
    cfg = load_config({"model": {"arch": args.arch, "dtype": "fp32"}, "particles": {"num": args.particles}})
    w = make_vit_weights(arch, seed=int(cfg["model"]["weights"]["seed"]))
    clip = synthetic_clip(2)
    ot = OracleTracker(cfg, w, arch)
    ot.init(clip[0], cfg["input"]["bbox0"])

    done = [0]
    t_start = [0.0]
    feats = ot.features

    def features_with_progress(frame, particles, chunk=None):
        out = []
        for i in range(0, particles.shape[1], 256):
            out.append(feats(frame, np.ascontiguousarray(particles[:, i:i + 256]), chunk or args.batch))
            done[0] += out[-1].shape[0]
            print(f"cpu_frame: {done[0]} / {particles.shape[1]} crops, {time.perf_counter() - t_start[0]:.1f} s",
                  file=sys.stderr, flush=True)
        return np.concatenate(out, 0)

    ot.features = features_with_progress
    t_start[0] = time.perf_counter()
    est = ot.track(clip[1])
    measured = time.perf_counter() - t_start[0]

    sample = bench.cpu_baseline(args.arch, args.particles, args.sample_seconds, threads)
    print(json.dumps({"measured_full_frame_s": round(measured, 2), "measured_frames_per_s": 1.0 / measured,
                      "estimate": est, "particles": args.particles, "arch": args.arch, "threads": threads,
                      "host_cpus": cpus, "bench_cpu_baseline": sample,
                      "extrapolation_over_measured": round(sample["s_per_frame"] / measured, 4)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
