"""`ParticleFilter` — the reference's "Particle Filter ... probabilistic algorithms for accurate state
estimation" (/root/reference/README.md:8), SPEC.md S2/S5-S7, on the HIP path.

Particles are sharded by index across ranks (rank r owns [r*P/G, (r+1)*P/G)); one process per GPU.
Per frame the only cross-device traffic is:

  1. an all-gather of each shard's 32-byte statistics {T_r (int64), sum Q*x, sum Q*y, sum Q*s (fp64)}.
     It provides the global weight normaliser T (the "weight-normalisation sum"), the shard offsets
     O_r = sum_{q<r} T_q that make the integer systematic resample exact and shard-invariant, and the
     estimate, summed in rank order so every rank computes the same bits;
  2. an all-gather of the resampled chunks (ancestor index + state, 16 B per slot, padded to the largest
     chunk) from which each rank keeps the slots it owns for the next frame.

Both run on torch.distributed (backend "nccl" = RCCL over xGMI on the GPU box; "gloo" in CPU tests of the
exchange logic). With G = 1 there is no collective.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import torch

from . import _lib
from . import ops  # noqa: F401

vpf = torch.ops.vpf

_M0, _M1, _W0, _W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
_MASK = 0xFFFFFFFF


def philox4x32_10(ctr: Sequence[int], key: Sequence[int]) -> List[int]:
    """Host Philox4x32-10 (SPEC S1) for the per-frame resample offset word."""
    c0, c1, c2, c3 = (int(v) & _MASK for v in ctr)
    k0, k1 = (int(v) & _MASK for v in key)
    for r in range(10):
        if r:
            k0, k1 = (k0 + _W0) & _MASK, (k1 + _W1) & _MASK
        p0, p1 = _M0 * c0, _M1 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & _MASK, p1 & _MASK, ((p0 >> 32) ^ c3 ^ k1) & _MASK, p0 & _MASK
    return [c0, c1, c2, c3]


def resample_word(seed: int, frame: int) -> int:
    seed &= (1 << 64) - 1
    return philox4x32_10((0, frame, 1, 0), (seed & _MASK, seed >> 32))[0]


def position(j: int, T: int, P: int, U: int) -> int:
    """SPEC S7: pos_j = floor((j*T + floor(U*T/2^32)) / P) (Python ints: exact)."""
    u = (U * T) >> 32
    return (j * T + u) // P


def slot_range(offset: int, shard_T: int, T: int, P: int, U: int) -> Tuple[int, int]:
    """Slots j whose position falls in [offset, offset + shard_T): a contiguous range (pos is monotone)."""
    def first_at_least(v: int) -> int:
        lo, hi = 0, P
        while lo < hi:
            mid = (lo + hi) // 2
            if position(mid, T, P, U) >= v:
                hi = mid
            else:
                lo = mid + 1
        return lo
    return first_at_least(offset), first_at_least(offset + shard_T)


def _all_gather_into(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """all_gather_into_tensor on the group's backend. RCCL ("nccl") takes the device tensors directly, on the
    current stream. gloo (CPU tests; several ranks sharing one GPU) exchanges host copies."""
    import torch.distributed as dist
    if inp.is_cuda and dist.get_backend(group) == "gloo":
        host = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(host, inp.cpu(), group=group)
        out.copy_(host)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)


def gather_stats(packed: torch.Tensor, world_size: int, group=None) -> List[Tuple[int, float, float, float]]:
    """All-gather each shard's packed int64[4] = {T_r, bits of sum Qx, sum Qy, sum Qs} and decode on the host.
    Works for any device / backend (RCCL on the GPU box, gloo on CPU)."""
    if world_size > 1:
        allp = torch.empty(world_size * 4, dtype=torch.int64, device=packed.device)
        _all_gather_into(allp, packed.contiguous().view(-1), group)
        allp = allp.view(world_size, 4)
    else:
        allp = packed.view(1, 4)
    host = allp.cpu()
    T_r = host[:, 0].tolist()
    sums = host[:, 1:].contiguous().view(torch.float64).tolist()
    return [(int(T_r[r]), *sums[r]) for r in range(world_size)]


def plan_resample(stats, P: int, n_local: int, U: int):
    """Host plan of the exact systematic resample (SPEC S7) from the gathered shard statistics:
    (uniform, T, offsets, slot ranges per rank)."""
    world = len(stats)
    T_r = [s[0] for s in stats]
    uniform = sum(T_r) == 0
    if uniform:
        T_r = [n_local] * world
    T = sum(T_r)
    offsets = [sum(T_r[:r]) for r in range(world)]
    ranges = [slot_range(offsets[r], T_r[r], T, P, U) for r in range(world)]
    return uniform, T, offsets, ranges


def exchange_chunks(chunk: torch.Tensor, ranges, begin: int, n_local: int, world_size: int, group=None):
    """All-gather the padded per-rank resample chunks ([4][cap] = x, y, s, ancestor bits) and keep the slots
    [begin, begin + n_local) this rank owns. Returns [4][n_local]."""
    cap = chunk.shape[1]
    allc = torch.empty(world_size * 4 * cap, device=chunk.device, dtype=chunk.dtype)
    _all_gather_into(allc, chunk.contiguous().view(-1), group)
    allc = allc.view(world_size, 4, cap)
    parts = []
    for r, (ra, rb) in enumerate(ranges):
        lo, hi = max(ra, begin), min(rb, begin + n_local)
        if lo < hi:
            parts.append(allc[r, :, lo - ra: hi - ra])
    return torch.cat(parts, dim=1)


class ParticleFilter:
    """H1, H10-H12. API: predict(), update(features, template), estimate(), resample(),
    attributes `particles` (float32[3][P_local] on the device, SoA rows x, y, scale) and `Q` (int64[P_local])."""

    def __init__(self, num_particles: int, init_state=(0.0, 0.0, 1.0), motion_std=(4.0, 4.0, 0.02),
                 scale_range=(0.5, 2.0), seed: int = 1234, device=None, frame_size=(224, 224),
                 lam: float = 20.0, weight_bits: int = 40, rank: int = 0, world_size: int = 1,
                 group: Optional[object] = None):
        if world_size < 1 or num_particles % world_size:
            raise ValueError("num_particles must be divisible by world_size")
        if weight_bits + max(1, (num_particles - 1).bit_length()) > 62:
            raise ValueError("weight_bits + ceil(log2 P) must be <= 62 (SPEC S5)")
        if not (math.isfinite(float(lam)) and float(lam) >= 0.0):
            raise ValueError("lam must be finite and >= 0 (SPEC S5)")
        self.P = int(num_particles)
        self.rank, self.world_size, self.group = int(rank), int(world_size), group
        self.n_local = self.P // self.world_size
        self.begin = self.rank * self.n_local
        self.motion_std = [float(v) for v in motion_std]
        self.scale_range = [float(v) for v in scale_range]
        self.seed = int(seed)
        self.lam, self.bits = float(lam), int(weight_bits)
        self.height, self.width = int(frame_size[0]), int(frame_size[1])
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.particles = torch.empty(3, self.n_local, device=self.device, dtype=torch.float32)
        self.Q = torch.zeros(self.n_local, device=self.device, dtype=torch.int64)
        self._T = torch.zeros(1, device=self.device, dtype=torch.int64)
        self._sums = torch.zeros(3, device=self.device, dtype=torch.float64)
        self._cdf = torch.empty(self.n_local, device=self.device, dtype=torch.int64)
        self._states = torch.empty(3, self.n_local, device=self.device, dtype=torch.float32)
        self._anc = torch.empty(self.n_local, device=self.device, dtype=torch.int32)
        self.frame = 0
        self.last_ancestors: Optional[torch.Tensor] = None
        self._stats_host: Optional[List[Tuple[int, float, float, float]]] = None
        self.reset(init_state)

    # ------------------------------------------------------------------ state
    def reset(self, state) -> None:
        x, y, s = (float(v) for v in state)
        self.particles[0].fill_(x)
        self.particles[1].fill_(y)
        self.particles[2].fill_(s)
        self.Q.zero_()
        self.frame = 0
        self._stats_host = None

    def predict(self, frame: Optional[int] = None) -> None:
        """H1: counter-based random walk (SPEC S2) for frame index `frame` (default: next frame)."""
        self.frame = self.frame + 1 if frame is None else int(frame)
        vpf.predict_(self.particles, self.begin, self.seed, self.frame, self.motion_std, float(self.width),
                     float(self.height), self.scale_range)
        self._stats_host = None

    def update(self, features: torch.Tensor, template: torch.Tensor) -> torch.Tensor:
        """H10 from explicit features [n][D] fp32 (LN'd CLS) and a unit template [D]: sets Q."""
        n, D = features.shape
        if n != self.n_local:
            raise ValueError(f"update: expected {self.n_local} feature rows, got {n}")
        vpf.cosine_weight(features.to(torch.float32).contiguous(), template.to(torch.float32).contiguous(),
                          self.lam, self.bits, self.Q, None)
        self._stats_host = None
        return self.Q

    def set_weights(self, Q: torch.Tensor) -> None:
        if Q.data_ptr() != self.Q.data_ptr():
            self.Q.copy_(Q)
        self._stats_host = None

    # ------------------------------------------------------------------ H11
    def _gather_stats(self) -> List[Tuple[int, float, float, float]]:
        if self._stats_host is None:
            vpf.shard_stats(self.Q, self.particles, self._T, self._sums)
            packed = torch.cat([self._T, self._sums.view(torch.int64)])          # 4 x int64 = 32 B
            self._stats_host = gather_stats(packed, self.world_size, self.group)
        return self._stats_host

    def estimate(self) -> Tuple[float, float, float]:
        """SPEC S6: weighted mean state; every rank returns the same bits (rank-order sums)."""
        st = self._gather_stats()
        T = sum(s[0] for s in st)
        if T == 0:
            m = self.particles.to(torch.float64).sum(dim=1)
            if self.world_size > 1:
                allm = torch.empty(self.world_size * 3, dtype=torch.float64, device=m.device)
                _all_gather_into(allm, m.contiguous(), self.group)
                m = allm.view(self.world_size, 3).sum(dim=0)
            m = (m / self.P).tolist()
            return float(m[0]), float(m[1]), float(m[2])
        sx = sy = ss = 0.0
        for s in st:
            sx += s[1]; sy += s[2]; ss += s[3]
        return sx / T, sy / T, ss / T

    # ------------------------------------------------------------------ H12
    def resample(self) -> torch.Tensor:
        """SPEC S7 systematic resample; returns the global ancestor indices of this rank's slots."""
        st = self._gather_stats()
        U = resample_word(self.seed, self.frame)
        uniform, T, offsets, ranges = plan_resample(st, self.P, self.n_local, U)
        a, b = ranges[self.rank]
        cnt = b - a
        if self.world_size == 1:
            vpf.resample(self.Q, self.begin, offsets[0], T, self.P, U, uniform, 0, self.P, self.particles, self._anc,
                         self._states, self._cdf)
            self.particles.copy_(self._states)
            self.last_ancestors = self._anc.clone()
        else:
            cap = max(1, max(r[1] - r[0] for r in ranges))
            chunk = torch.zeros(4, cap, device=self.device, dtype=torch.float32)
            if cnt > 0:
                anc_c = torch.empty(cnt, device=self.device, dtype=torch.int32)
                states_c = torch.empty(3, cnt, device=self.device, dtype=torch.float32)
                vpf.resample(self.Q, self.begin, offsets[self.rank], T, self.P, U, uniform, a, b, self.particles,
                             anc_c, states_c, self._cdf)
                chunk[:3, :cnt] = states_c
                chunk[3, :cnt] = anc_c.view(torch.float32)
            new = exchange_chunks(chunk, ranges, self.begin, self.n_local, self.world_size, self.group)
            self.particles.copy_(new[:3])
            self.last_ancestors = new[3].contiguous().view(torch.int32)
        self.Q.zero_()
        self._stats_host = None
        return self.last_ancestors
