"""Headline benchmark: frames/s of the full per-frame tracking step at 4096 particles, ViT-B/16 @ 224,
bf16 (BASELINE.json metric / configs[1]); 1/2/4/8 MI355X by sharding the same 4096 particles (strong
scaling: the metric is quoted at a fixed particle count).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = one frame: predict -> crop + ViT-B/16 forward (HIP graph replay) -> weights -> estimate ->
resample (+ RCCL all-gathers when N > 1). Frames (synthetic u8 224x224, moving textured target) are
resident in HBM before the timed region. Rank 0 prints ONE JSON line. Extra fields:
  roofline      the dominant kernel (the FC1 GEMM by default: the largest FLOP share) timed by HIP events on
                its own stream in an eager pass after the timed region: achieved TFLOP/s vs the 2.5 PF dense
                bf16 MFMA peak (MI355X_MICROARCH.md). traffic = HBM bytes per launch of that kernel from the
                newest committed PMC summary profiles/r<N>_pmc_traffic.json (tools/gpu_session.sh pmc), when taken on
                this workload; else null.
  frame_mfma_frac  whole-frame algorithmic FLOPs (35.126 GFLOP/crop) x fps / peak.
  kernels       per-kernel-type HIP-event averages from the same eager pass.
  cpu_baseline  the CPU oracle (torch fp32 ViT + C particle-filter ops, "port": the reference has no
                runnable code) timed on this host's cores: ONE full tracking frame at the workload's particle count
                (OracleTracker.track after a warm-up batch; ~160-190 s for 4096 particles on 16 cores), with the
                bounded crop-sample extrapolation of earlier rounds beside it as a cross-check (rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/sec @ 4096 particles, ViT-B/16 224px; 1/2/4/8 MI355X scaling"
PEAK_BF16_TFLOPS = 2500.0     # dense bf16 MFMA, /opt/skills/guides/MI355X_MICROARCH.md (Matrix cores)
PEAK_FP8_TFLOPS = 5000.0      # dense block-scaled e4m3 MFMA (same table), the fp8 path's GEMMs


# newest committed PMC summary first (profiles/r<round>_pmc_traffic[_<dtype>][_<tag>].json)
def _pmc_files(dtype: str):
    import glob
    import re
    suffix = "" if dtype == "bf16" else f"_{dtype}"
    out = []
    for path in glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_traffic{suffix}*.json")):
        m = re.match(rf"r(\d+)_pmc_traffic{suffix}(_[a-z0-9]+)?\.json$", os.path.basename(path))
        if m and (dtype != "bf16" or not (m.group(2) or "").startswith("_fp")):
            out.append((int(m.group(1)), path))
    return [p for _, p in sorted(out, reverse=True)]


def pmc_traffic(arch_name: str, n_local: int, kernel: str, dtype: str = "bf16", frame=None):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary (tools/pmc_traffic.py over two rocprofv3
    passes of this bench: FETCH_SIZE x2 gfx950 correction + WRITE_SIZE) taken on the same workload (arch, particles
    per GPU, dtype, and the source frame when the summary records it); otherwise (None, reason)."""
    for path in _pmc_files(dtype):
        try:
            with open(path) as f:
                d = json.load(f)
            if (d.get("arch") != arch_name or int(d.get("particles_per_gpu", -1)) != n_local
                    or d.get("dtype", "bf16") != dtype
                    or (frame is not None and d.get("frame") not in (None, list(frame)))):
                continue
            k = d["kernels"][kernel]
            return int(k["traffic_bytes"]), os.path.relpath(path, ROOT)
        except (OSError, KeyError, ValueError):
            continue
    return None, "no PMC summary for this workload"


# BASELINE.json configs as presets (global particle count, arch, dtype, frame). configs[0] is the reference's
# CPU-runnable plumbing case (its CPU path is oracle/, timed as cpu_baseline); on the GPU it is ViT-Ti.
PRESETS = {
    0: dict(particles=256, arch="vit_tiny_patch16_224", dtype="bf16", frame="224x224"),
    1: dict(particles=4096, arch="vit_base_patch16_224", dtype="bf16", frame="224x224"),
    2: dict(particles=16384, arch="vit_base_patch16_224", dtype="bf16", frame="224x224"),
    3: dict(particles=4096, arch="vit_large_patch14_336", dtype="bf16", frame="224x224"),
    4: dict(particles=65536, arch="vit_base_patch16_224", dtype="fp8", frame="1080x1920"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", type=int, choices=sorted(PRESETS), default=None,
                    help="BASELINE.json configs[i] (sets --particles/--arch/--dtype/--frame; the metric's own "
                         "workload is configs[1], the default). configs[2]/[4] are 8-GPU sizes: with fewer ranks "
                         "use --particles for the per-GPU share")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--particles", type=int, default=4096, help="global particle count")
    ap.add_argument("--arch", default="vit_base_patch16_224")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8", "fp32"],
                    help="fp8: MX-fp8 QKV / FC1 / FC2 GEMMs (configs[4])")
    ap.add_argument("--frame", default="224x224", help="synthetic source frame HxW (configs[4]: 1080x1920)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for N > 1: nccl (= RCCL over xGMI, the product path) or gloo "
                         "(host-staged; lets several ranks share one GPU to rehearse the multi-rank path)")
    ap.add_argument("--dist-timeout", type=float, default=120.0,
                    help="seconds: bound on the process-group rendezvous and on any collective (RCCL watchdog), so "
                         "a broken multi-GPU start fails fast and names its rank (vpf.distributed)")
    ap.add_argument("--kernel-frames", type=int, default=2, help="eager frames timed per kernel (roofline)")
    ap.add_argument("--cpu-frame-budget", type=float, default=480.0,
                    help="seconds: a full CPU frame projected above this falls back to the bounded sample")
    ap.add_argument("--cpu-baseline", default="full", choices=["full", "sample", "off"],
                    help="full: time one whole oracle frame (value) + the bounded sample (cross-check); sample: the "
                         "bounded-sample extrapolation only; off: skip")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="bounded-sample budget (s); 0 = no sample")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = host_cpus() rule: the affinity set, capped by a cgroup quota and OMP_NUM_THREADS, and "
                         "at 16 when neither is set")
    args = ap.parse_args()
    if args.preset is not None:
        given = {a.lstrip("-").split("=")[0].replace("-", "_") for a in sys.argv[1:] if a.startswith("--")}
        for k, v in PRESETS[args.preset].items():
            if k not in given:          # explicit flags win over the preset
                setattr(args, k, v)
    return args


CPU_THREAD_CAP = 16   # the GPU box's CPU share per GPU (cgroup quota 16, OMP_NUM_THREADS=16): the rounds-1-2 default


def host_cpus():
    """The host's CPU model and the cores this process may use: its affinity set, capped by a cgroup CPU quota
    and by OMP_NUM_THREADS when the launcher sets one (the GPU box's CPU share: it sets 16 per GPU); with neither,
    capped at CPU_THREAD_CAP so the baseline's thread count is the same on every host."""
    info = {"affinity": len(os.sched_getaffinity(0)), "cgroup_quota": None, "omp_num_threads": None, "model": None}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    info["model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                info["cgroup_quota"] = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        info["omp_num_threads"] = int(os.environ["OMP_NUM_THREADS"])
    use = info["affinity"]
    if info["cgroup_quota"]:
        use = min(use, max(1, int(info["cgroup_quota"])))
    if info["omp_num_threads"]:
        use = min(use, info["omp_num_threads"])
    if not info["cgroup_quota"] and not info["omp_num_threads"]:
        use = min(use, CPU_THREAD_CAP)
    info["threads"] = use
    info["thread_rule"] = (f"min(affinity, cgroup quota, OMP_NUM_THREADS); {CPU_THREAD_CAP} when neither quota nor "
                           "OMP_NUM_THREADS is set")
    return info


def cpu_baseline(arch_name: str, P: int, budget_s: float, threads: int):
    """Oracle CPU path (the reference's "CPU path": oracle/, torch fp32 ViT + the C particle-filter ops) on a bounded
    sample of the same workload: crops of the metric's frame through the fp32 ViT for ~budget_s, then the PF ops at the
    full P. One frame = P crops + the PF ops, so s/frame = (measured s per crop) x P + PF time: a linear extrapolation in
    the crop count (the oracle runs crops in independent batches of 8), checked by one separately timed full frame
    (tools/cpu_frame.py, profiles/r3_cpu_full_frame.log)."""
    import numpy as np
    import torch

    from oracle import pf as opf
    from oracle import vit as ovit
    from vitparticlefiltertracker_amd.config import ARCHS
    from vitparticlefiltertracker_amd.frames import synthetic_clip
    from vitparticlefiltertracker_amd.weights import make_vit_weights

    arch = ARCHS[arch_name]
    cpus = host_cpus()
    threads = threads or cpus["threads"]
    torch.set_num_threads(threads)
    w = make_vit_weights(arch, seed=0)
    frame = synthetic_clip(2)[1]
    rng = np.random.default_rng(0)
    batch = 8
    part = np.empty((3, batch), np.float32)
    part[0], part[1], part[2] = rng.uniform(90, 130, batch), rng.uniform(90, 130, batch), rng.uniform(0.8, 1.2, batch)
    # warm-up
    patches = opf.crop_patches(frame, part, (64.0, 64.0), arch.img_size, arch.patch, arch.patch_kp, (0.5,) * 3, (0.5,) * 3)
    ovit.features_from_patches(torch.from_numpy(patches), w, arch)
    crops, t0, per_batch = 0, time.perf_counter(), []
    while time.perf_counter() - t0 < budget_s:
        tb = time.perf_counter()
        patches = opf.crop_patches(frame, part, (64.0, 64.0), arch.img_size, arch.patch, arch.patch_kp, (0.5,) * 3,
                                   (0.5,) * 3)
        ovit.features_from_patches(torch.from_numpy(patches), w, arch)
        per_batch.append(time.perf_counter() - tb)
        crops += batch
    # the median batch: the box's 16-CPU share is noisy (co-tenants), and a mean over 15 s took one interference burst
    # as 22 % of extra time against a separately timed full frame (profiles/r3_cpu_full_frame.log)
    t_vit = float(np.median(per_batch)) / batch
    t_vit_mean = (time.perf_counter() - t0) / crops
    # particle-filter ops at the full P (predict, estimate, resample)
    pp = np.empty((3, P), np.float32)
    pp[0], pp[1], pp[2] = 112.0, 112.0, 1.0
    Q = rng.integers(0, 1 << 40, P, dtype=np.int64)
    t1 = time.perf_counter()
    opf.predict(pp, 0, 1234, 1, (4.0, 4.0, 0.02), 224, 224, (0.5, 2.0))
    opf.estimate(Q, pp)
    opf.resample(Q, 12345)
    t_pf = time.perf_counter() - t1
    s_per_frame = t_vit * P + t_pf
    return {"value": 1.0 / s_per_frame, "unit": "frames/s", "cores": threads, "kind": "port",
            "cpu_model": cpus["model"],
            "host_cpus": {k: cpus[k] for k in ("affinity", "cgroup_quota", "omp_num_threads", "thread_rule")},
            "s_per_frame": round(s_per_frame, 2), "s_per_crop": round(t_vit, 5),
            "s_per_crop_mean": round(t_vit_mean, 5), "pf_ops_s": round(t_pf, 5),
            "extrapolation": f"s/frame = median s/crop (per batch of {batch}) x {P} crops + PF ops at P={P} (linear in "
                             f"crops: independent batches; one full frame timed separately: "
                             f"profiles/r3_cpu_full_frame.log)",
            "sample": f"{crops} crops of {arch_name} fp32 (torch CPU oracle, batch {batch}) in "
                      f"{t_vit * crops:.1f} s + PF ops at P={P}; extrapolated to one {P}-particle frame "
                      f"({s_per_frame:.1f} s/frame)"}


def cpu_full_frame(arch_name: str, P: int, threads: int, sample_s: float, budget_s: float = 480.0):
    """cpu_baseline: ONE full tracking frame of the CPU oracle at the workload's particle
    count, measured: OracleTracker.init on frame 0, a warm-up batch, then OracleTracker.track on frame 1 (predict, P
    crops through the fp32 ViT in batches of 8, weights, estimate, resample), wall clock. Progress to stderr every 512
    crops. With sample_s > 0 the bounded-sample extrapolation (cpu_baseline above) runs after it as a cross-check.
    A 32-crop probe after the warm-up projects the frame first; above budget_s (a slow host, or a workload such as
    ViT-L/14 or 8192 particles whose CPU frame takes many minutes) the bounded sample alone is reported, marked as such,
    so that bench.py still finishes within a few minutes."""
    import numpy as np
    import torch

    from oracle.tracker import OracleTracker
    from vitparticlefiltertracker_amd.config import ARCHS, load_config
    from vitparticlefiltertracker_amd.frames import synthetic_clip
    from vitparticlefiltertracker_amd.weights import make_vit_weights

    arch = ARCHS[arch_name]
    cpus = host_cpus()
    threads = threads or cpus["threads"]
    torch.set_num_threads(threads)
    cfg = load_config({"model": {"arch": arch_name, "dtype": "fp32"}, "particles": {"num": P}})
    w = make_vit_weights(arch, seed=int(cfg["model"]["weights"]["seed"]))
    clip = synthetic_clip(2)
    ot = OracleTracker(cfg, w, arch)
    ot.init(clip[0], cfg["input"]["bbox0"])
    ot.features(clip[1], np.ascontiguousarray(ot.particles[:, :8]), 8)        # warm-up batch
    tp = time.perf_counter()                                                   # projection probe: 4 batches of 8
    ot.features(clip[1], np.ascontiguousarray(ot.particles[:, :32]), 8)
    projected = (time.perf_counter() - tp) / 32 * P
    if projected > budget_s:   # a slow host or a big workload: keep bench.py's wall time bounded, say so
        x = cpu_baseline(arch_name, P, max(sample_s, 15.0), threads)
        x["measured"] = (f"bounded sample: the full frame was projected at {projected:.0f} s (32-crop probe), over the "
                         f"{budget_s:.0f}-s budget (--cpu-frame-budget)")
        return x
    feats, done, t0 = ot.features, [0], [0.0]

    def features_with_progress(frame, particles, chunk=None):
        out = []
        for i in range(0, particles.shape[1], 512):
            out.append(feats(frame, np.ascontiguousarray(particles[:, i:i + 512]), 8))
            done[0] += out[-1].shape[0]
            print(f"bench.py cpu_baseline: {done[0]} / {particles.shape[1]} crops, {time.perf_counter() - t0[0]:.1f} s",
                  file=sys.stderr, flush=True)
        return np.concatenate(out, 0)

    ot.features = features_with_progress
    t0[0] = time.perf_counter()
    ot.track(clip[1])
    measured = time.perf_counter() - t0[0]
    out = {"value": 1.0 / measured, "unit": "frames/s", "cores": threads, "kind": "port",
           "cpu_model": cpus["model"],
           "host_cpus": {k: cpus[k] for k in ("affinity", "cgroup_quota", "omp_num_threads", "thread_rule")},
           "s_per_frame": round(measured, 2), "measured": "full frame",
           "sample": f"one full {P}-particle tracking frame of the CPU oracle (OracleTracker.track: predict, {P} crops "
                     f"of {arch_name} fp32 through the torch CPU ViT in batches of 8, weights, estimate, resample), "
                     f"after a warm-up batch: {measured:.1f} s"}
    if sample_s > 0:
        try:
            x = cpu_baseline(arch_name, P, sample_s, threads)
            out["cross_check"] = {k: x[k] for k in ("s_per_frame", "s_per_crop", "s_per_crop_mean", "pf_ops_s",
                                                    "sample")}
            out["cross_check"]["extrapolated_over_measured"] = round(x["s_per_frame"] / measured, 4)
        except Exception as e:  # report, never fake
            out["cross_check"] = {"error": repr(e)}
    return out


def main() -> int:
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dist_backend == "gloo":
        local = local % max(1, torch.cuda.device_count())     # ranks may share a GPU (rehearsal only)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        # bounded rendezvous + one probe collective, rank / world / backend on stderr first
        from vitparticlefiltertracker_amd.distributed import init_distributed
        init_distributed(args.dist_backend, dev if args.dist_backend == "nccl" else None, args.dist_timeout, rank,
                         world)
    if args.particles < world:
        raise SystemExit("--particles must be at least the number of ranks")
    if args.gpus != world and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch N > 1 ranks with "
              "python -m torch.distributed.run --nproc-per-node N ... (measuring the ranks that exist)", file=sys.stderr)

    from vitparticlefiltertracker_amd import Tracker, load_config
    from vitparticlefiltertracker_amd.config import ARCHS
    from vitparticlefiltertracker_amd.frames import synthetic_clip
    from vitparticlefiltertracker_amd.vit import KernelTimer

    cfg = load_config({"model": {"arch": args.arch, "dtype": args.dtype}, "particles": {"num": args.particles}})
    arch = ARCHS[args.arch]
    n_frames = 1 + args.warmup + args.steps + args.kernel_frames
    fh, fw = (int(v) for v in args.frame.lower().split("x"))
    clip = synthetic_clip(n_frames, fh, fw)
    frames = [torch.from_numpy(f).to(dev) for f in clip]          # resident in HBM before timing
    tr = Tracker(cfg, device=dev, rank=rank, world_size=world, use_graph=not args.no_graph)
    tr.init(frames[0], cfg["input"]["bbox0"])
    for k in range(args.warmup):
        tr.track(frames[1 + k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        tr.track(frames[1 + args.warmup + k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    fps = args.steps / elapsed

    # per-kernel HIP-event timing in eager mode on the same buffers / stream (after the timed region)
    timer = KernelTimer()
    tr.engine.timer = timer
    use_graph = tr.use_graph
    tr.use_graph = False
    base = 1 + args.warmup + args.steps
    for k in range(args.kernel_frames):
        tr.track(frames[base + k])
    tr.use_graph = use_graph
    tr.engine.timer = None
    ks = timer.summary()
    n_loc = tr.n_local   # rank 0's shard (floor(P / N) particles when N does not divide P)
    M = n_loc * arch.tokens
    D, F = arch.dim, arch.mlp
    flops = {"gemm_fc1": 2.0 * M * D * F, "gemm_fc2": 2.0 * M * F * D, "gemm_qkv": 2.0 * M * D * 3 * D,
             "gemm_proj": 2.0 * M * D * D, "gemm_patch": 2.0 * n_loc * arch.n_patches * arch.patch_k * D,
             "attention": 2.0 * 2.0 * n_loc * arch.heads * arch.tokens ** 2 * arch.head_dim}
    for name, v in ks.items():
        if name in flops:
            v["tflops"] = flops[name] / (v["avg_ms"] * 1e-3) / 1e12
    dom = max((n for n in flops if n.startswith("gemm") and n in ks), key=lambda n: ks[n]["total_ms"])
    ach = ks[dom]["tflops"]
    traffic, traffic_src = (pmc_traffic(args.arch, n_loc, dom, args.dtype, (fh, fw)) if args.dtype in ("bf16", "fp8")
                            else (None, None))
    # the dominant GEMM's MFMA peak: dense bf16, or dense MX-fp8 for the fp8 path's block-scaled GEMMs
    peak = PEAK_FP8_TFLOPS if args.dtype == "fp8" and dom in ("gemm_qkv", "gemm_fc1", "gemm_fc2") else PEAK_BF16_TFLOPS
    gflop_frame = arch.gflop_per_crop() * args.particles
    gflop_exec = arch.gflop_per_crop_executed(cls_fused=tr.engine.cls_fused) * args.particles
    gflop_mx8 = arch.gflop_per_crop_mx8() * args.particles if args.dtype == "fp8" else 0.0

    def frame_peak_time(gflop, gflop8):
        """Seconds the frame's MFMA work takes at the dense peaks (gflop8 of it on MX8 GEMMs)."""
        return (gflop8 / PEAK_FP8_TFLOPS + (gflop - gflop8) / PEAK_BF16_TFLOPS) * 1e9 / 1e12
    check = multi_rank_check(tr, world, rank, dev, args.dist_backend) if world > 1 else None
    line = {
        "metric": METRIC,
        "value": round(fps, 4),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": {"bf16": "bf16", "fp32": "f32", "fp8": "fp8-e4m3(MX)+bf16"}[args.dtype],
        "data": f"synthetic: u8 {fh}x{fw} frames (uniform-noise background, moving 64x64 textured target), "
                "seeded random-init ViT weights (no pretrained checkpoint offline)",
        "config": {"workload": f"{args.particles} particles, {args.arch} {args.dtype}, {fh}x{fw} frames, "
                               "full tracking step per frame",
                   "particles": args.particles, "particles_per_gpu": n_loc, "arch": args.arch, "frame": [fh, fw],
                   "hip_graph": not args.no_graph, "parallelism": f"particle-shard x{world}",
                   **({"dist_backend": dist.get_backend(), "dist_world_size": dist.get_world_size()}
                      if world > 1 else {}),
                   **({"dist_note": "gloo: ranks may share a GPU (rehearsal, not a product number)"}
                      if world > 1 and args.dist_backend == "gloo" else {})},
        "roofline": {"bound": "mfma", "kernel": dom, "achieved": round(ach, 2), "peak": peak,
                     "unit": "TFLOP/s", "frac": round(ach / peak, 4), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "avg_launch_ms": round(ks[dom]["avg_ms"], 4),
                     "flop_per_launch": flops[dom]},
        # full-forward FLOPs (SURVEY §8d's count, what the metric's roofline is quoted on) and the FLOPs of the work
        # the product actually performs (the last block computes the CLS row only; config.gflop_per_crop_executed),
        # each as the fraction of the frame the MFMA work would take at its dense peak: the fp8 path's block-scaled
        # GEMMs against the fp8 peak, everything else against bf16 (frame_peak_note; VERDICT r4 #6: round 4 divided the
        # fp8 frame's FLOPs by the bf16 peak alone, which overstated its utilisation ~2x)
        "frame_mfma_frac": round(fps * frame_peak_time(gflop_frame, gflop_mx8) / world, 4),
        "frame_mfma_frac_executed": round(fps * frame_peak_time(gflop_exec, gflop_mx8) / world, 4),
        "frame_peak_note": ("bf16 dense peak" if gflop_mx8 == 0 else
                            f"FLOP-weighted: {round(gflop_mx8 / args.particles, 4)} GFLOP per crop of MX8 GEMMs at "
                            f"{PEAK_FP8_TFLOPS:.0f} TF, the rest at {PEAK_BF16_TFLOPS:.0f} TF"),
        "gflop_per_crop": {"full_forward": round(arch.gflop_per_crop(), 4),
                           "executed": round(gflop_exec / args.particles, 4)},
        "kernels": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                    for k, v in ks.items()},
        **({"multi_rank_check": check} if check is not None else {}),
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and args.cpu_baseline != "off":
        try:
            if args.cpu_baseline == "full":
                line["cpu_baseline"] = cpu_full_frame(args.arch, args.particles, args.cpu_threads, args.cpu_seconds,
                                                      args.cpu_frame_budget)
            elif args.cpu_seconds > 0:
                line["cpu_baseline"] = cpu_baseline(args.arch, args.particles, args.cpu_seconds, args.cpu_threads)
        except Exception as e:  # report, never fake
            line["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if check is not None and not check["ok"]:
        print(f"bench.py: the ranks disagree: {json.dumps(check)}", file=sys.stderr, flush=True)
        return 1
    return 0


def multi_rank_check(tr, world: int, rank: int, dev, backend: str):
    """N > 1 self-check of the last timed frame (the driver's scaling run proves itself): the backend and world size
    the process group reports; every rank's estimate bits; a checksum of the global CDF every rank computed from the
    all-gathered weights (identical iff every rank saw the same global weights); each rank's ancestor range, which
    must tile the global systematic resample in rank order (ancestors are non-decreasing in the slot index)."""
    import struct

    import torch
    import torch.distributed as dist
    pf = tr.pf
    est = pf._read_estimate()
    cdf = pf._cdf.to(torch.int64)
    mix = torch.arange(1, 2 * cdf.numel(), 2, device=cdf.device, dtype=torch.int64)
    cdf_sum = int((cdf * mix).sum().item())              # wraps mod 2^64: a checksum, not a value
    anc = pf.last_ancestors
    mine = [float(v) for v in est] + [cdf_sum, int(cdf[-1].item()), int(anc[0].item()), int(anc[-1].item()),
                                      int((anc[1:] >= anc[:-1]).all().item()), int(anc.numel())]
    t = torch.tensor([struct.unpack("<q", struct.pack("<d", v))[0] if i < 3 else v for i, v in enumerate(mine)],
                     dtype=torch.int64, device=dev if backend == "nccl" else "cpu")
    out = torch.empty(world * t.numel(), dtype=torch.int64, device=t.device)
    dist.all_gather_into_tensor(out, t)
    rows = out.view(world, -1).cpu().tolist()
    est_bits = [tuple(r[:3]) for r in rows]
    ok_est = all(e == est_bits[0] for e in est_bits)
    ok_cdf = all(r[3] == rows[0][3] and r[4] == rows[0][4] for r in rows)
    ok_anc = all(r[7] == 1 for r in rows) and all(rows[i][6] <= rows[i + 1][5] for i in range(world - 1))
    ok_cnt = sum(r[8] for r in rows) == pf.P
    return {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "estimates_agree": ok_est,
            "cdf_checksum_agree": ok_cdf, "ancestors_sorted_across_ranks": ok_anc, "slots_cover_P": ok_cnt,
            "estimate": [struct.unpack("<d", struct.pack("<q", v))[0] for v in est_bits[0]],
            "ok": ok_est and ok_cdf and ok_anc and ok_cnt}


if __name__ == "__main__":
    sys.exit(main())
