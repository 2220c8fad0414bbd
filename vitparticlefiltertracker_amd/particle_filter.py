"""`ParticleFilter` — the reference's "Particle Filter ... probabilistic algorithms for accurate state
estimation" (/root/reference/README.md:8), SPEC.md S2/S5-S7, on the HIP path.

Particles are sharded by index across ranks (rank r owns [floor(r*P/G), floor((r+1)*P/G)); shards
differ by at most one particle when G does not divide P); one process per GPU.
Per frame the only cross-device traffic is ONE fixed-size all-gather of the shard chunks (weight Q_i int64 +
state x, y, s fp32 = 20 B per particle; 80 KB at 4096 particles, 1.3 MB at configs[4]'s 65536; every chunk is sized
for the largest shard). Every rank then holds the global weights and states, and one device call
(vpf_estimate_resample) computes on each rank:

  * the weight-normalisation sum T and the estimate sums (SPEC S6), in one fixed-order tree over the GLOBAL
    index, so every rank and every world size gets the same bits;
  * the inclusive CDF and, from the resample word drawn on the device, the exact systematic-resample ancestors
    of the slots this rank owns (SPEC S7): identical to the single-process oracle for any G.

No host planning sits between the weights and the resample; the host reads only the 32-B statistics (the
estimate it returns). The collective runs on torch.distributed (backend "nccl" = RCCL over xGMI on the GPU box;
"gloo" in CPU tests of the layout and when several ranks share one GPU). With G = 1 there is no collective.
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


def shard_range(P: int, world: int, rank: int) -> Tuple[int, int]:
    """(begin, n) of rank `rank`'s particles: [floor(rank P / world), floor((rank + 1) P / world)).
    Equal shards when world divides P; otherwise the sizes differ by one. Needs 1 <= world <= P."""
    if not 1 <= world <= P or not 0 <= rank < world:
        raise ValueError(f"need 1 <= world_size <= particles and 0 <= rank < world_size (P={P}, world={world}, "
                         f"rank={rank})")
    b, e = rank * P // world, (rank + 1) * P // world
    return b, e - b


def plan_resample(stats, P: int, n_local, U: int):
    """Host plan of the exact systematic resample (SPEC S7) for the per-shard entry point vpf_resample, from the
    shards' (T_r, ...) statistics: (uniform, T, offsets, slot ranges per rank). `n_local`: the shard size (equal
    shards) or the list of shard sizes. ParticleFilter itself runs the device-resident vpf_estimate_resample and
    needs no plan."""
    world = len(stats)
    T_r = [s[0] for s in stats]
    uniform = sum(T_r) == 0
    if uniform:
        T_r = list(n_local) if isinstance(n_local, (list, tuple)) else [n_local] * world
    T = sum(T_r)
    offsets = [sum(T_r[:r]) for r in range(world)]
    ranges = [slot_range(offsets[r], T_r[r], T, P, U) for r in range(world)]
    return uniform, T, offsets, ranges


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


def chunk_words(n: int) -> int:
    """int32 words of one shard chunk: Q int64[n] | x | y | s fp32[n], padded to a multiple of 8 bytes."""
    return 5 * n + (n & 1)


def shard_views(chunk: torch.Tensor, n: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """(Q int64[n], particles f32[3][n]) as views into one shard chunk (int32[chunk_words(n)]): the filter's
    state lives in the chunk, so the all-gather sends it as is (no packing)."""
    return chunk[: 2 * n].view(torch.int64), chunk[2 * n: 5 * n].view(torch.float32).view(3, n)


def global_view(allc: torch.Tensor, world: int, n: int):
    """Kernel arguments of vpf_estimate_resample for `world` gathered chunks of n particles each (allc:
    int32[world * chunk_words(n)]): (Q view, q_stride, particle view, ld, p_stride, n_shard)."""
    cw = chunk_words(n)
    return allc.view(torch.int64), cw // 2, allc[2 * n:].view(torch.float32), n, cw, n


def compact_index(P: int, world: int) -> torch.Tensor:
    """Unequal shards (world does not divide P): int32-word indices into the gathered chunks (world slots of
    chunk_words(ceil(P / world)) words; rank r's slot holds its shard_views layout for its own n_r) that read out
    the global arrays in particle order: Q int64[P] as 2P words, then x | y | s fp32[P]. One index_select of the
    gathered buffer with it gives the one-shard layout that vpf_estimate_resample reads as (Q, P, x|y|s, P, 3P, P)."""
    cw = chunk_words(-(-P // world))
    q, st = [], [[], [], []]
    for r in range(world):
        _, n = shard_range(P, world, r)
        base = r * cw
        q.append(torch.arange(base, base + 2 * n))
        for c in range(3):
            st[c].append(torch.arange(base + (2 + c) * n, base + (3 + c) * n))
    return torch.cat(q + st[0] + st[1] + st[2])


def compact_view(glob: torch.Tensor, P: int):
    """vpf_estimate_resample's arguments over the compacted global arrays (glob: int32[5P], compact_index order)."""
    return glob[: 2 * P].view(torch.int64), P, glob[2 * P:].view(torch.float32), P, 3 * P, P


class ParticleFilter:
    """H1, H10-H12. API: predict(), update(features, template), estimate(), resample(),
    attributes `particles` (float32[P_local][3] on the device: one (x, y, scale) row per particle, §8b's shape) and
    `Q` (int64[P_local]). The storage is SoA, `particles_soa` (float32[3][P_local]); `particles` is its transposed view.

    `Q` and `particles_soa` are views into one shard chunk (`shard_views`). Per frame (`step`, or estimate() then
    resample()): world > 1 all-gathers the chunks (20 B per particle, one fixed-size RCCL collective), then ONE
    device call, vpf_estimate_resample, computes the estimate sums, the CDF, the resample word and the ancestors
    of this rank's slots over the global set. The resample is enqueued before the host waits for the 32-B
    statistics, so the only host synchronisation of a frame is that read."""

    def __init__(self, num_particles: int, init_state=(0.0, 0.0, 1.0), motion_std=(4.0, 4.0, 0.02),
                 scale_range=(0.5, 2.0), seed: int = 1234, device=None, frame_size=(224, 224),
                 lam: float = 20.0, weight_bits: int = 40, rank: int = 0, world_size: int = 1,
                 group: Optional[object] = None):
        self.begin, self.n_local = shard_range(int(num_particles), int(world_size), int(rank))
        if weight_bits + max(1, (num_particles - 1).bit_length()) > 62:
            raise ValueError("weight_bits + ceil(log2 P) must be <= 62 (SPEC S5)")
        if not (math.isfinite(float(lam)) and float(lam) >= 0.0):
            raise ValueError("lam must be finite and >= 0 (SPEC S5)")
        self.P = int(num_particles)
        self.rank, self.world_size, self.group = int(rank), int(world_size), group
        n = self.n_local
        n_max = -(-self.P // self.world_size)     # every rank's chunk has the largest shard's size (fixed-size gather)
        self.motion_std = [float(v) for v in motion_std]
        self.scale_range = [float(v) for v in scale_range]
        self.seed = int(seed)
        self.lam, self.bits = float(lam), int(weight_bits)
        self.height, self.width = int(frame_size[0]), int(frame_size[1])
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._chunk = torch.zeros(chunk_words(n_max), device=self.device, dtype=torch.int32)
        self.Q, self.particles_soa = shard_views(self._chunk, n)
        self._cidx = None
        if self.world_size > 1:
            self._allc = torch.zeros(self.world_size * chunk_words(n_max), device=self.device, dtype=torch.int32)
            if self.P % self.world_size == 0:
                self._gview = global_view(self._allc, self.world_size, n)
            else:   # unequal shards: the gathered chunks are compacted into the global order first (_settle)
                self._cidx = compact_index(self.P, self.world_size).to(self.device)
                self._glob = torch.empty(5 * self.P, device=self.device, dtype=torch.int32)
                self._gview = compact_view(self._glob, self.P)
        else:
            self._gview = (self.Q, n, self.particles_soa.view(-1), n, 3 * n, n)
        self._cdf = torch.empty(self.P, device=self.device, dtype=torch.int64)
        self._states = torch.empty(3, n, device=self.device, dtype=torch.float32)
        self._anc = torch.empty(n, device=self.device, dtype=torch.int32)
        self._stats_dev = torch.zeros(4, device=self.device, dtype=torch.int64)
        self._stats_pin = torch.zeros(4, dtype=torch.int64).pin_memory()
        self._stats_evt = torch.cuda.Event()
        self.frame = 0
        self.last_ancestors: Optional[torch.Tensor] = None
        self._settled = False                                   # estimate / resample of the current Q computed
        self._est: Optional[Tuple[float, float, float]] = None  # its host value once read
        self.reset(init_state)

    # ------------------------------------------------------------------ state
    @property
    def particles(self) -> torch.Tensor:
        """The particles as float32[P_local][3] rows (x, y, scale): SURVEY.md §8b's `.particles [P, 3]`, so
        `particles[:, 0]` is every particle's x. A transposed VIEW of the SoA storage `particles_soa` (float32[3][P_local],
        the layout the kernels and the all-gathered chunk use); writes through it land in the filter's state."""
        return self.particles_soa.t()

    @particles.setter
    def particles(self, value) -> None:
        """Assign [P_local][3] states (x, y, scale per row): copied into the SoA storage."""
        v = torch.as_tensor(value, dtype=torch.float32, device=self.device)
        if tuple(v.shape) != (self.n_local, 3):
            raise ValueError(f"particles: expected shape ({self.n_local}, 3), got {tuple(v.shape)}")
        self.particles_soa.copy_(v.t())
        self._settled = False

    @property
    def states(self) -> torch.Tensor:
        """Alias of `particles` ([P_local][3] view)."""
        return self.particles_soa.t()

    def reset(self, state) -> None:
        x, y, s = (float(v) for v in state)
        self.particles_soa[0].fill_(x)
        self.particles_soa[1].fill_(y)
        self.particles_soa[2].fill_(s)
        self.Q.zero_()
        self.frame = 0
        self._settled = False

    def predict(self, frame: Optional[int] = None) -> None:
        """H1: counter-based random walk (SPEC S2) for frame index `frame` (default: next frame)."""
        self.frame = self.frame + 1 if frame is None else int(frame)
        vpf.predict_(self.particles_soa, self.begin, self.seed, self.frame, self.motion_std, float(self.width),
                     float(self.height), self.scale_range)
        self._settled = False

    def update(self, features: torch.Tensor, template: torch.Tensor) -> torch.Tensor:
        """H10 from explicit features [n][D] fp32 (LN'd CLS) and a unit template [D]: sets Q."""
        n, D = features.shape
        if n != self.n_local:
            raise ValueError(f"update: expected {self.n_local} feature rows, got {n}")
        vpf.cosine_weight(features.to(torch.float32).contiguous(), template.to(torch.float32).contiguous(),
                          self.lam, self.bits, self.Q, None)
        self._settled = False
        return self.Q

    def set_weights(self, Q: torch.Tensor) -> None:
        if Q.data_ptr() != self.Q.data_ptr():
            self.Q.copy_(Q)
        self._settled = False

    # ------------------------------------------------------------------ H11 + H12 on the device
    def _settle(self) -> None:
        """Enqueue (world > 1: the chunk all-gather, then) vpf_estimate_resample for the current weights and the
        32-B statistics' copy to pinned host memory. No host synchronisation."""
        if self._settled:
            return
        if self.world_size > 1:
            _all_gather_into(self._allc, self._chunk, self.group)
            if self._cidx is not None:
                torch.index_select(self._allc, 0, self._cidx, out=self._glob)
        Qv, qs, Pv, ld, ps, nsh = self._gview
        vpf.estimate_resample(Qv, qs, Pv, ld, ps, nsh, self.P, self.seed, self.frame, self.begin,
                              self.begin + self.n_local, self._anc, self._states, self._cdf, self._stats_dev)
        self._stats_pin.copy_(self._stats_dev, non_blocking=True)
        self._stats_evt.record()
        self._settled = True
        self._est = None

    def _commit(self) -> None:
        """Enqueue the resample computed by _settle: this rank's slots take their ancestors' states."""
        self.particles_soa.copy_(self._states)
        self.last_ancestors = self._anc.clone()
        self.Q.zero_()
        self._settled = False

    def _read_estimate(self) -> Tuple[float, float, float]:
        """SPEC S6 from the settled statistics (waits for their D2H copy): sum Q*state / T, or the plain mean
        when T == 0. The sums are the same bits on every rank and for every world size."""
        if self._est is None:
            self._stats_evt.synchronize()
            T = int(self._stats_pin[0])
            sx, sy, ss = self._stats_pin[1:].view(torch.float64).tolist()
            d = float(T) if T else float(self.P)
            self._est = (sx / d, sy / d, ss / d)
        return self._est

    def estimate(self) -> Tuple[float, float, float]:
        """SPEC S6: weighted mean state of the current particles and weights."""
        self._settle()
        return self._read_estimate()

    def resample(self) -> torch.Tensor:
        """SPEC S7 systematic resample; returns the global ancestor indices of this rank's slots."""
        self._settle()
        self._commit()
        return self.last_ancestors

    def step(self) -> Tuple[float, float, float]:
        """estimate() then resample() of one frame, with the resample enqueued before the host waits for the
        estimate (Tracker.track)."""
        self._settle()
        self._commit()
        return self._read_estimate()
