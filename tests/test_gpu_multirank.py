"""GPU (one MI355X): the multi-rank Tracker on real HIP kernels. Two ranks share cuda:0 and exchange through
gloo (host-staged all-gathers; the GPU box has one GPU, so RCCL cannot pair two ranks on it). Everything
else is the product path: per-shard crop + ViT + weights on the device, vpf_shard_stats, the exact
systematic-resample plan, vpf_resample on each rank's slot range and the chunk exchange.
The sharded run must reproduce the single-rank Tracker's ancestors and particle states bit for bit, give the
same estimate bits on every rank, and match the single-rank estimate to 1e-12 (fp64 summation order)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

P, FRAMES = 256, 5


def _cfg():
    from vitparticlefiltertracker_amd import load_config
    return load_config({"model": {"arch": "vit_tiny_patch16_224", "dtype": "bf16", "weights": {"seed": 3}},
                        "particles": {"num": P, "seed": 99}})


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(tr, clip):
    out = []
    tr.init(clip[0], (80, 80, 64, 64))
    for f in clip[1:]:
        est = tr.track(f)
        out.append((est, tr.pf.last_ancestors.cpu().numpy().copy(), tr.pf.particles.cpu().numpy().copy()))
    return out


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vitparticlefiltertracker_amd import Tracker
        from vitparticlefiltertracker_amd.frames import synthetic_clip
        tr = Tracker(_cfg(), device="cuda:0", rank=rank, world_size=world)
        q.put((rank, _run(tr, synthetic_clip(FRAMES + 1))))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_tracker_equals_single_rank(world):
    from vitparticlefiltertracker_amd import Tracker
    from vitparticlefiltertracker_amd.frames import synthetic_clip
    ref = _run(Tracker(_cfg(), device="cuda:0"), synthetic_clip(FRAMES + 1))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = P // world
    for r in range(world):
        assert not isinstance(out[r], str), out[r]
        for k, ((est, anc, parts), (est1, anc1, parts1)) in enumerate(zip(out[r], ref), start=1):
            # the estimate's fp64 partial sums are combined per shard, then in rank order: identical bits on
            # every rank of one run (checked below), and equal to the single-rank value up to summation order
            np.testing.assert_allclose(est, est1, rtol=1e-12, atol=0, err_msg=f"rank {r} frame {k}")
            assert np.array_equal(anc, anc1[r * n:(r + 1) * n]), f"rank {r} frame {k}: ancestors"
            assert np.array_equal(parts.view(np.uint32), parts1[:, r * n:(r + 1) * n].view(np.uint32)), \
                f"rank {r} frame {k}: particle states"
    for k in range(FRAMES):
        assert all(out[r][k][0] == out[0][k][0] for r in range(world)), f"frame {k + 1}: ranks disagree"
