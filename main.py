"""`python main.py [--config config.yaml]` — the entry point the reference documents (README.md:34-38):
read the config, feed frames to the Tracker, print the tracked positions (README.md:42).

Several targets (README.md:46-50, SPEC S9): `input.bboxes: [[x, y, w, h], ...]` runs a MultiTracker (one batched ViT
pass over every target's particles); each frame then prints and records one position per target, --video-out
draws every box, and --checkpoint / --resume save and restore every target.

Multi-GPU: `torchrun --nproc-per-node G --master-addr 127.0.0.1 main.py` shards the particles over G GPUs.
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys
import time


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--config", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "config.yaml"))
    ap.add_argument("--frames", type=int, default=None, help="override input.frames")
    ap.add_argument("--out", default=None, help="write positions as JSON here")
    ap.add_argument("--video-out", default=None,
                    help="write the frames with the tracked box drawn: a .y4m file, or a directory of frames")
    ap.add_argument("--frame-format", default="ppm", choices=["ppm", "png", "jpg"],
                    help="image format of the --video-out directory's frames (png / jpg through Pillow)")
    ap.add_argument("--checkpoint", default=None,
                    help="save the tracker state (np.savez; per rank with several GPUs) here after the last frame")
    ap.add_argument("--checkpoint-every", type=int, default=0, help="also save every N frames")
    ap.add_argument("--resume", default=None,
                    help="continue from a checkpoint: the source's frames up to its frame index are skipped")
    ap.add_argument("--dist-timeout", type=float, default=120.0,
                    help="seconds: bound on the multi-GPU rendezvous and on any collective (vpf.distributed)")
    args = ap.parse_args(argv)

    import torch
    import torch.distributed as dist
    from vitparticlefiltertracker_amd import MultiTracker, Tracker, load_config
    from vitparticlefiltertracker_amd.frames import Y4MWriter, draw_box, iter_frames, prefetch, synthetic_clip

    cfg = load_config(args.config)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 and not dist.is_initialized():
        from vitparticlefiltertracker_amd.distributed import init_distributed
        dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        torch.cuda.set_device(dev)
        # RCCL bound to this rank's GPU eagerly (device_id), a bounded rendezvous and one probe collective (as bench.py)
        init_distributed("nccl", dev, args.dist_timeout)
    inp = cfg["input"]
    n = args.frames or int(inp["frames"])
    if inp["source"] == "synthetic":
        src = iter_frames(synthetic_clip(n, inp["height"], inp["width"], tuple(inp["bbox0"]), inp["seed"]))
    else:
        src = itertools.islice(iter_frames(inp["source"]), n)
    frames = prefetch(src, depth=2)   # decode + pin on a host thread, overlapped with the GPU frame loop
    boxes = inp.get("bboxes")
    if boxes is not None:
        return _run_multi(args, cfg, boxes, frames, MultiTracker, dist)
    tr = Tracker(cfg)
    first = next(frames)
    start = 1
    if args.resume:
        tr.load_checkpoint(args.resume)
        for _ in range(tr.frame_index):       # frames 1 .. frame_index were tracked before the checkpoint
            if next(frames, None) is None:
                raise SystemExit(f"--resume: the checkpoint is at frame {tr.frame_index}, past the end of the input")
        start = tr.frame_index + 1
    else:
        tr.init(first, inp["bbox0"])
    sink = None
    if args.video_out and tr.rank == 0:
        if args.video_out.lower().endswith(".y4m"):
            sink = Y4MWriter(args.video_out)
        else:
            os.makedirs(args.video_out, exist_ok=True)

    def emit(k, rgb, box):
        if not args.video_out or tr.rank != 0:
            return
        img = draw_box(rgb.numpy() if hasattr(rgb, "numpy") else rgb, box)
        if sink is not None:
            sink.write(img)
        else:
            _write_frame(args, k, img)

    if not args.resume:
        emit(0, first, inp["bbox0"])
    t0 = time.perf_counter()
    out = []
    for k, f in enumerate(frames, start=start):
        x, y, s = tr.track(f)
        out.append({"frame": k, "x": x, "y": y, "scale": s})
        emit(k, f, tr.box((x, y, s)))
        if tr.rank == 0:
            print(f"frame {k:4d}  x={x:8.2f}  y={y:8.2f}  scale={s:6.3f}", flush=True)
        if args.checkpoint and args.checkpoint_every > 0 and k % args.checkpoint_every == 0:
            tr.save_checkpoint(args.checkpoint)
    if args.checkpoint:
        tr.save_checkpoint(args.checkpoint)
    if sink is not None:
        sink.close()
    dt = time.perf_counter() - t0
    if tr.rank == 0:
        print(f"{len(out)} frames in {dt:.3f} s ({len(out) / max(dt, 1e-9):.2f} frames/s)", file=sys.stderr)
        if args.out:
            with open(args.out, "w") as fh:
                json.dump(out, fh, indent=1)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


def _sink(args, rank):
    """(emit(k, rgb, boxes), close()) for --video-out: the frame with every box drawn, as .y4m or image frames."""
    from vitparticlefiltertracker_amd.frames import Y4MWriter, draw_box
    if not args.video_out or rank != 0:
        return (lambda k, rgb, boxes: None), (lambda: None)
    writer = Y4MWriter(args.video_out) if args.video_out.lower().endswith(".y4m") else None
    if writer is None:
        os.makedirs(args.video_out, exist_ok=True)

    def emit(k, rgb, boxes):
        img = rgb.numpy() if hasattr(rgb, "numpy") else rgb
        for b in boxes:
            img = draw_box(img, b)
        if writer is not None:
            writer.write(img)
        else:
            _write_frame(args, k, img)
    return emit, (writer.close if writer is not None else (lambda: None))


def _write_frame(args, k, img) -> None:
    """Frame k of a --video-out directory in --frame-format (PPM with numpy; PNG / JPEG through Pillow)."""
    from vitparticlefiltertracker_amd.frames import write_image_pil, write_ppm
    path = os.path.join(args.video_out, f"frame_{k:05d}.{args.frame_format}")
    if args.frame_format == "ppm":
        write_ppm(path, img)
    else:
        write_image_pil(path, img)


def _run_multi(args, cfg, boxes, frames, MultiTracker, dist) -> int:
    """input.bboxes: K targets tracked by one MultiTracker; one line and one JSON record per frame with every
    target's (x, y, scale)."""
    mt = MultiTracker(cfg, n_objects=len(boxes))
    first = next(frames)
    start = 1
    if args.resume:
        mt.load_checkpoint(args.resume)
        for _ in range(mt.frame_index):       # frames 1 .. frame_index were tracked before the checkpoint
            if next(frames, None) is None:
                raise SystemExit(f"--resume: the checkpoint is at frame {mt.frame_index}, past the end of the input")
        start = mt.frame_index + 1
    else:
        mt.init(first, boxes)
    emit, close = _sink(args, mt.rank)
    if not args.resume:
        emit(0, first, boxes)
    t0 = time.perf_counter()
    out = []
    for k, f in enumerate(frames, start=start):
        ests = mt.track(f)
        out.append({"frame": k, "targets": [{"x": x, "y": y, "scale": s} for x, y, s in ests]})
        # the box sizes being tracked (restored from the checkpoint after --resume), not the config's
        emit(k, f, [_box(st, (0.0, 0.0, w, h)) for st, (w, h) in zip(ests, mt.boxes)])
        if mt.rank == 0:
            print(f"frame {k:4d}  " + "  ".join(f"[{i}] x={x:8.2f} y={y:8.2f} s={s:6.3f}"
                                                 for i, (x, y, s) in enumerate(ests)), flush=True)
        if args.checkpoint and args.checkpoint_every > 0 and k % args.checkpoint_every == 0:
            mt.save_checkpoint(args.checkpoint)
    if args.checkpoint:
        mt.save_checkpoint(args.checkpoint)
    close()
    dt = time.perf_counter() - t0
    if mt.rank == 0:
        print(f"{len(out)} frames x {len(boxes)} targets in {dt:.3f} s ({len(out) / max(dt, 1e-9):.2f} frames/s)",
              file=sys.stderr)
        if args.out:
            with open(args.out, "w") as fh:
                json.dump(out, fh, indent=1)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


def _box(state, bbox0):
    """(x, y, w, h) of a state (centre, scale) for a target whose frame-0 box is bbox0 (SPEC S3)."""
    x, y, s = (float(v) for v in state)
    w, h = s * float(bbox0[2]), s * float(bbox0[3])
    return x - 0.5 * w, y - 0.5 * h, w, h


if __name__ == "__main__":
    sys.exit(main())
