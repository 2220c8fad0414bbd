"""GPU (one MI355X): the multi-rank Tracker on real HIP kernels. Two ranks share cuda:0 and exchange through
gloo (host-staged all-gathers; the GPU box has one GPU, so RCCL cannot pair two ranks on it). Everything
else is the product path: per-shard crop + ViT + weights on the device, the all-gather of the shard chunks and
vpf_estimate_resample over the global set on every rank. The sharded run must reproduce the
single-rank Tracker's estimates, ancestors and particle states bit for bit on every rank."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

FRAMES = 5


def _cfg(P):
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
        out.append((est, tr.pf.last_ancestors.cpu().numpy().copy(), tr.pf.particles_soa.cpu().numpy().copy()))
    return out


def _worker(rank, world, port, P, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vitparticlefiltertracker_amd import Tracker
        from vitparticlefiltertracker_amd.frames import synthetic_clip
        tr = Tracker(_cfg(P), device="cuda:0", rank=rank, world_size=world)
        q.put((rank, _run(tr, synthetic_clip(FRAMES + 1))))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,P", [(2, 256), (4, 256), (3, 33), (3, 100)])
def test_sharded_tracker_equals_single_rank(world, P):
    """(3, 33): 11 particles per rank, an odd (padded) shard chunk and a world size that is not a power of two.
    (3, 100): unequal shards (33 / 33 / 34; SURVEY.md §8e's [floor(rP/G), floor((r+1)P/G)) ranges), compacted into the
    global order after the gather."""
    from vitparticlefiltertracker_amd.particle_filter import shard_range
    from vitparticlefiltertracker_amd import Tracker
    from vitparticlefiltertracker_amd.frames import synthetic_clip
    ref = _run(Tracker(_cfg(P), device="cuda:0"), synthetic_clip(FRAMES + 1))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, P, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert not isinstance(out[r], str), out[r]
        b, n = shard_range(P, world, r)
        for k, ((est, anc, parts), (est1, anc1, parts1)) in enumerate(zip(out[r], ref), start=1):
            # every rank sums the gathered global set in one fixed order: the single-rank estimate's bits
            assert est == est1, f"rank {r} frame {k}: estimate {est} vs single rank {est1}"
            assert np.array_equal(anc, anc1[b:b + n]), f"rank {r} frame {k}: ancestors"
            assert np.array_equal(parts.view(np.uint32), parts1[:, b:b + n].view(np.uint32)), \
                f"rank {r} frame {k}: particle states"
    for k in range(FRAMES):
        assert all(out[r][k][0] == out[0][k][0] for r in range(world)), f"frame {k + 1}: ranks disagree"


# ------------------------------------------------------------------ MultiTracker across ranks (§8f rank 4)
BOXES = [(40, 50, 48, 48), (120, 100, 56, 40)]


def _mt_cfg(P, dtype="bf16", alpha=0.0):
    from vitparticlefiltertracker_amd import load_config
    return load_config({"model": {"arch": "vit_tiny_patch16_224", "dtype": dtype, "weights": {"seed": 3}},
                        "particles": {"num": P, "seed": 99}, "likelihood": {"template_update": alpha}})


def _mt_run(mt, clip):
    """Per frame: every target's estimate, this rank's weights (before the resample), ancestors and states."""
    out = []
    mt.init(clip[0], BOXES)
    for f in clip[1:]:
        mt._upload(f)
        mt.frame_index += 1
        for pf in mt.pfs:
            pf.height, pf.width = int(f.shape[0]), int(f.shape[1])
            pf.predict(mt.frame_index)
        mt.weigh()
        Qs = [pf.Q.cpu().numpy().copy() for pf in mt.pfs]
        ests = mt.step()
        out.append((ests, [pf.last_ancestors.cpu().numpy().copy() for pf in mt.pfs],
                    [pf.particles_soa.cpu().numpy().copy() for pf in mt.pfs], Qs))
    return out


def _mt_worker(rank, world, port, P, dtype, alpha, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vitparticlefiltertracker_amd import MultiTracker
        from vitparticlefiltertracker_amd.frames import synthetic_clip
        mt = MultiTracker(_mt_cfg(P, dtype, alpha), n_objects=len(BOXES), device="cuda:0", rank=rank, world_size=world)
        q.put((rank, _mt_run(mt, synthetic_clip(FRAMES + 1))))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _mt_sharded(world, P, dtype="bf16", alpha=0.0):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mt_worker, args=(r, world, port, P, dtype, alpha, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert not isinstance(out[r], str), out[r]
    return out


@pytest.mark.parametrize("world,P,alpha", [(2, 128, 0.0), (3, 33, 0.5), (2, 45, 0.5)])
def test_sharded_multitracker_equals_single_rank_and_oracle(world, P, alpha):
    """Two targets with different boxes, each target's particles sharded over the ranks (bf16):
    * every rank returns the single-rank MultiTracker's estimates bit for bit, and its shards of every target's
      weights, ancestors and states;
    * against the oracle directly: the ranks' weight shards, concatenated in rank order, injected into
      OracleMultiTracker give every rank's ancestors and states bit for bit and the estimates to 1e-12, every frame.
    (3, 33): 11 particles per rank per target, odd shard chunks; alpha = 0.5: the template update on every rank.
    (2, 45): unequal shards (22 / 23 per target)."""
    from oracle.tracker import OracleMultiTracker
    from vitparticlefiltertracker_amd.particle_filter import shard_range
    from vitparticlefiltertracker_amd import MultiTracker
    from vitparticlefiltertracker_amd.config import ARCHS
    from vitparticlefiltertracker_amd.frames import synthetic_clip
    from vitparticlefiltertracker_amd.weights import make_vit_weights
    cfg = _mt_cfg(P, "bf16", alpha)
    clip = synthetic_clip(FRAMES + 1)
    ref = _mt_run(MultiTracker(cfg, n_objects=len(BOXES), device="cuda:0"), clip)
    out = _mt_sharded(world, P, "bf16", alpha)
    K = len(BOXES)
    sl = [slice(b, b + n) for b, n in (shard_range(P, world, r) for r in range(world))]
    for r in range(world):
        for k, ((ests, ancs, parts, Qs), (ests1, ancs1, parts1, Qs1)) in enumerate(zip(out[r], ref), start=1):
            assert ests == ests1, f"rank {r} frame {k}: estimates {ests} vs single rank {ests1}"
            for t in range(K):
                assert np.array_equal(Qs[t], Qs1[t][sl[r]]), f"rank {r} frame {k} target {t}: weights"
                assert np.array_equal(ancs[t], ancs1[t][sl[r]]), f"rank {r} frame {k} target {t}"
                assert np.array_equal(parts[t].view(np.uint32), parts1[t][:, sl[r]].view(np.uint32))
    arch = ARCHS["vit_tiny_patch16_224"]
    om = OracleMultiTracker(cfg, K, make_vit_weights(arch, seed=3), arch)
    om.init(clip[0], BOXES)
    for k in range(FRAMES):
        Qg = [np.concatenate([out[r][k][3][t] for r in range(world)]) for t in range(K)]
        e_ref = om.track(clip[k + 1], Qg)
        for r in range(world):
            for t in range(K):
                np.testing.assert_allclose(out[r][k][0][t], e_ref[t], rtol=1e-12)
                assert np.array_equal(out[r][k][1][t], om.targets[t].last_ancestors[sl[r]]), (r, k, t)
                assert np.array_equal(out[r][k][2][t].view(np.uint32),
                                      om.targets[t].particles[:, sl[r]].view(np.uint32)), (r, k, t)


def test_sharded_multitracker_fp32_matches_oracle():
    """Two ranks, two targets, fp32 parity mode with a template update: every rank's per-target estimates within 1e-4
    relative of OracleMultiTracker's own (no injection), per frame."""
    from oracle.tracker import OracleMultiTracker
    from vitparticlefiltertracker_amd.config import ARCHS
    from vitparticlefiltertracker_amd.frames import synthetic_clip
    from vitparticlefiltertracker_amd.weights import make_vit_weights
    world, P = 2, 64
    cfg = _mt_cfg(P, "fp32", 0.5)
    clip = synthetic_clip(FRAMES + 1)
    out = _mt_sharded(world, P, "fp32", 0.5)
    arch = ARCHS["vit_tiny_patch16_224"]
    om = OracleMultiTracker(cfg, len(BOXES), make_vit_weights(arch, seed=3), arch)
    om.init(clip[0], BOXES)
    for k in range(FRAMES):
        e_ref = om.track(clip[k + 1])
        for r in range(world):
            assert out[r][k][0] == out[0][k][0]
            for t in range(len(BOXES)):
                np.testing.assert_allclose(np.array(out[r][k][0][t]), np.array(e_ref[t]), rtol=1e-4,
                                           err_msg=f"rank {r} frame {k + 1} target {t}")
