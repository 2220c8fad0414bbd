"""CPU, world_size 2 and 8 (gloo): the multi-rank exchange of ParticleFilter — statistics all-gather, exact
resample plan, chunk all-gather and slot ownership — reproduces the single-process oracle bit for bit
(SURVEY.md §8e). The per-shard device work (vpf_shard_stats / vpf_resample) is emulated by the oracle here;
the GPU tests cover those kernels against the same oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import pf
from vitparticlefiltertracker_amd import particle_filter as PF


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, P, seed, frames, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _body(rank, world, P, seed, frames, q)
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _body(rank, world, P, seed, frames, q):
    if True:
        rng = np.random.default_rng(seed)
        n = P // world
        begin = rank * n
        parts = np.empty((3, P), np.float32)
        parts[0], parts[1], parts[2] = 100.0, 90.0, 1.0
        ref = parts.copy()
        local = np.ascontiguousarray(parts[:, begin:begin + n])
        results = []
        for k in range(1, frames + 1):
            # identical global weights on every rank; each rank uses only its shard
            Q = rng.integers(0, 1 << 40, P, dtype=np.int64)
            if k == 2:
                Q[:] = 0                                  # T == 0 -> uniform fallback path
            if k == 3:
                Q[rng.random(P) < 0.9] = 0
            pf.predict(local, begin, 77, k, (3.0, 3.0, 0.05), 224, 224, (0.5, 2.0))
            pf.predict(ref, 0, 77, k, (3.0, 3.0, 0.05), 224, 224, (0.5, 2.0))
            Ql = np.ascontiguousarray(Q[begin:begin + n])
            T_r, sums = pf.shard_stats(Ql, local)
            packed = torch.cat([torch.tensor([T_r], dtype=torch.int64),
                                torch.from_numpy(sums.copy()).view(torch.int64)])
            stats = PF.gather_stats(packed, world)
            T = sum(s[0] for s in stats)
            est = (sum(s[1] for s in stats) / T, sum(s[2] for s in stats) / T, sum(s[3] for s in stats) / T) if T else None
            U = PF.resample_word(77, k)
            uniform, Tt, offsets, ranges = PF.plan_resample(stats, P, n, U)
            a, b = ranges[rank]
            Quse = np.ones(n, np.int64) if uniform else Ql
            C = np.cumsum(Quse)
            cap = max(1, max(r1 - r0 for r0, r1 in ranges))
            chunk = torch.zeros(4, cap, dtype=torch.float32)
            for jj, j in enumerate(range(a, b)):
                li = int(np.searchsorted(C, PF.position(j, Tt, P, U) - offsets[rank], side="right"))
                chunk[:3, jj] = torch.from_numpy(local[:, li].copy())
                chunk[3, jj] = torch.tensor([begin + li], dtype=torch.int32).view(torch.float32)
            new = PF.exchange_chunks(chunk, ranges, begin, n, world)
            local = np.ascontiguousarray(new[:3].numpy())
            anc_local = new[3].contiguous().view(torch.int32).numpy()
            # single-process oracle
            ref_est = pf.estimate(Q, ref)
            anc_ref = pf.resample(Q, pf.resample_U(77, k))
            ref = np.ascontiguousarray(ref[:, anc_ref])
            results.append((est, ref_est if T else None, np.array_equal(anc_local, anc_ref[begin:begin + n]),
                            np.array_equal(local, ref[:, begin:begin + n])))
        q.put((rank, results))


@pytest.mark.parametrize("world", [2, 8])
def test_two_rank_exchange_matches_oracle(world):
    """world 2, and world 8 (the driver's 8-GPU layout at 4096 particles: 512 per rank; here 64 per rank)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    P, frames = 512, 5
    procs = [ctx.Process(target=_worker, args=(r, world, port, P, 3, frames, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert not isinstance(out[r], str), out[r]
        for k, (est, ref_est, anc_ok, states_ok) in enumerate(out[r], start=1):
            assert anc_ok, f"rank {r} frame {k}: ancestors differ from the global oracle"
            assert states_ok, f"rank {r} frame {k}: states differ"
            if ref_est is not None:
                np.testing.assert_allclose(est, ref_est, rtol=1e-12)
    # every rank computes the same estimate bits
    for k in range(frames):
        for r in range(1, world):
            assert out[0][k][0] == out[r][k][0]
