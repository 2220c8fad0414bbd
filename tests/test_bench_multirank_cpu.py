"""CPU, world_size 2 and 4 (gloo): bench.py's N > 1 self-check (`multi_rank_check`), the part of the driver's
scaling run that proves the ranks saw one global weight set and agree on the estimate and the resample. Each rank
holds a stand-in filter (the attributes the check reads: the estimate, the global CDF it computed, its ancestor
slots) built from one shared global weight vector; the check must pass when they are consistent and fail when a
rank's estimate, CDF or ancestor range disagrees.

Also the fail-fast start of the N > 1 path (`vitparticlefiltertracker_amd/distributed.py`, used by
bench.py and main.py): on gloo, the bounded timeout is passed, the probe collective runs, rank / world / backend are
printed before anything blocks, and a rank whose partner never arrives fails within the timeout, naming itself."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _FakePF:
    """The attributes multi_rank_check reads, for rank r of `world` over P particles."""

    def __init__(self, rank, world, P, fault):
        rng = np.random.default_rng(7)
        Q = rng.integers(0, 1 << 30, P, dtype=np.int64)
        cdf = np.cumsum(Q)
        n = P // world
        slots = np.arange(rank * n, (rank + 1) * n)
        pos = (slots * cdf[-1]) // P                         # systematic positions, then ancestors (sorted)
        anc = np.searchsorted(cdf, pos, side="right")
        self.P = P
        self._cdf = torch.from_numpy(cdf.copy())
        self.last_ancestors = torch.from_numpy(anc.astype(np.int32))
        self._est = (111.25, 97.5, 1.0078125)
        if fault == "estimate" and rank == world - 1:
            self._est = (111.25, 97.5 + 2 ** -40, 1.0078125)   # one ulp-scale difference in y
        if fault == "cdf" and rank == world - 1:
            self._cdf[3] += 1
        if fault == "ancestors" and rank == world - 1:
            self.last_ancestors = self.last_ancestors.flip(0)    # not sorted

    def _read_estimate(self):
        return self._est


class _FakeTracker:
    def __init__(self, pf):
        self.pf = pf


def _worker(rank, world, port, P, fault, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    from vitparticlefiltertracker_amd.distributed import init_distributed
    init_distributed("gloo", None, 30.0, rank, world)     # what bench.py does at N > 1 (bounded, probed)
    try:
        import bench
        res = bench.multi_rank_check(_FakeTracker(_FakePF(rank, world, P, fault)), world, rank, "cpu", "gloo")
        q.put((rank, res))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _run(world, P, fault):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, P, fault, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert not isinstance(out[r], str), out[r]
    return out


@pytest.mark.parametrize("world", [2, 4])
def test_multi_rank_check_agrees(world):
    out = _run(world, 64, None)
    for r, res in out.items():
        assert res["ok"] and res["world_size"] == world and res["backend"] == "gloo", (r, res)
        assert res["estimate"] == [111.25, 97.5, 1.0078125]


@pytest.mark.parametrize("fault,flag", [("estimate", "estimates_agree"), ("cdf", "cdf_checksum_agree"),
                                        ("ancestors", "ancestors_sorted_across_ranks")])
def test_multi_rank_check_detects_disagreement(fault, flag):
    out = _run(2, 64, fault)
    for r, res in out.items():                             # every rank reaches the same verdict
        assert not res["ok"] and not res[flag], (r, res)


def test_cpu_full_frame_measures_or_falls_back_within_budget():
    """bench.py's cpu_baseline: a measured full oracle frame, or, when a 32-crop probe projects the frame past
    --cpu-frame-budget, the bounded sample marked as such (never an unmarked extrapolation)."""
    import bench
    full = bench.cpu_full_frame("vit_tiny_patch16_224", 48, 2, 0.0, budget_s=480.0)
    assert full["measured"] == "full frame" and full["s_per_frame"] > 0 and full["cores"] == 2
    assert abs(full["value"] * full["s_per_frame"] - 1.0) < 0.02
    fb = bench.cpu_full_frame("vit_tiny_patch16_224", 48, 2, 1.0, budget_s=1e-6)
    assert fb["measured"].startswith("bounded sample") and fb["s_per_frame"] > 0 and fb["kind"] == "port"


def _init_worker(rank, world, port, timeout_s, q):
    import contextlib
    import io
    import time
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    from vitparticlefiltertracker_amd.distributed import init_distributed
    err = io.StringIO()
    t0 = time.perf_counter()
    try:
        with contextlib.redirect_stderr(err):
            r, w, probe_ms = init_distributed("gloo", None, timeout_s, rank, world)
        q.put((rank, {"ok": True, "world": w, "probe_ms": probe_ms, "stderr": err.getvalue()}))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, {"ok": False, "error": repr(e), "seconds": time.perf_counter() - t0, "stderr": err.getvalue()}))


def _run_init(world, started, timeout_s):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_init_worker, args=(r, world, port, timeout_s, q)) for r in range(started)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    return out


def test_init_distributed_gloo_prints_and_probes():
    out = _run_init(2, 2, 30.0)
    for r, res in out.items():
        assert res["ok"] and res["world"] == 2, (r, res)
        assert f"rank {r} / world 2, backend gloo" in res["stderr"] and "timeout 30 s" in res["stderr"]
        assert "probe all_reduce" in res["stderr"] and res["probe_ms"] >= 0.0


def test_init_distributed_missing_rank_fails_within_timeout():
    """World 2 with only rank 0 started: the rendezvous gives up after the bounded timeout (3 s here, 120 s in
    bench.py) instead of torch's default, and the failure line names the rank, world and backend."""
    out = _run_init(2, 1, 3.0)
    res = out[0]
    assert not res["ok"] and res["seconds"] < 30.0, res
    assert "FAILED" in res["stderr"] and "rank 0 / world 2, backend gloo" in res["stderr"], res
