"""Process-group start for the particle-sharded path, shared by `bench.py`, `main.py` and
`tools/rccl_probe.py`: one process per GPU, RCCL (the "nccl" backend) over xGMI in the product, gloo for CPU
rehearsals.

The first RCCL run across GPUs is the driver's 8-GPU scaling bench, so a broken rendezvous or
RCCL/xGMI path must end that run quickly and say where instead of sitting at torch's 10-minute
default. `init_distributed`:
  * prints rank, world size, backend, device and the timeout to stderr before anything can block;
  * passes a bounded `timeout` to `init_process_group` (it bounds the TCP-store rendezvous and, for RCCL, the
    watchdog that aborts a hung collective);
  * runs one probe collective (a 1-element all-reduce of ones, expected = world size) on the backend's device, so the
    communicator is proven before the tracker allocates anything, and prints its result and time.
A wrong probe sum raises; a rendezvous that does not complete within the timeout raises from torch.
"""
from __future__ import annotations

import datetime
import os
import sys
import time

DEFAULT_TIMEOUT_S = 120.0


def _say(msg: str) -> None:
    print(f"[vpf.distributed] {msg}", file=sys.stderr, flush=True)


def init_distributed(backend: str, device=None, timeout_s: float = DEFAULT_TIMEOUT_S, rank=None, world_size=None):
    """Start the default process group for `backend` ("nccl" = RCCL, or "gloo") and prove it with one collective.

    `device`: this rank's torch.device (required for "nccl": the communicator is bound to it eagerly via device_id).
    `rank` / `world_size`: taken from RANK / WORLD_SIZE when None (the torchrun environment). Returns
    (rank, world_size, probe_ms)."""
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0")) if rank is None else int(rank)
    world_size = int(os.environ.get("WORLD_SIZE", "1")) if world_size is None else int(world_size)
    if backend == "nccl" and device is None:
        raise ValueError("init_distributed: the nccl (RCCL) backend needs this rank's device")
    where = (f"rank {rank} / world {world_size}, backend {backend}, device {device}, "
             f"master {os.environ.get('MASTER_ADDR', '?')}:{os.environ.get('MASTER_PORT', '?')}, timeout {timeout_s:g} s")
    _say(f"init_process_group: {where}")
    kw = {"timeout": datetime.timedelta(seconds=float(timeout_s)), "rank": rank, "world_size": world_size}
    if backend == "nccl":
        kw["device_id"] = device
    t0 = time.perf_counter()
    try:
        dist.init_process_group(backend, **kw)
    except Exception as e:
        _say(f"init_process_group FAILED after {time.perf_counter() - t0:.1f} s ({where}): {e!r}")
        raise
    t1 = time.perf_counter()
    probe = torch.ones(1, dtype=torch.float32, device=device if backend == "nccl" else "cpu")
    dist.all_reduce(probe)
    got = float(probe.item())            # waits for the collective (RCCL: the watchdog bounds it by the timeout)
    probe_ms = 1e3 * (time.perf_counter() - t1)
    if got != float(world_size):
        raise RuntimeError(f"init_distributed: probe all_reduce gave {got}, expected {world_size} ({where})")
    _say(f"ready: rank {rank} / world {dist.get_world_size()}, backend {dist.get_backend()}; rendezvous "
         f"{1e3 * (t1 - t0):.0f} ms, probe all_reduce {probe_ms:.1f} ms")
    return rank, world_size, probe_ms
