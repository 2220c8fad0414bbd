"""The ParticleFilter's chunk all-gather + vpf_estimate_resample through RCCL ("nccl" backend), one rank per GPU,
against a single-rank filter on the same weights: estimates, ancestors and states must be bit-identical.
torchrun --nproc-per-node G --master-addr 127.0.0.1 tools/rccl_probe.py   (needs G GPUs: RCCL refuses two ranks on
one device, "Duplicate GPU detected", profiles/r2_rccl_one_gpu_probe.txt)"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    from vitparticlefiltertracker_amd.distributed import init_distributed
    init_distributed("nccl", torch.device("cuda", dev), 120.0, rank, world)
    x = torch.full((4,), rank + 1, device="cuda", dtype=torch.int32)
    out = torch.empty(4 * world, device="cuda", dtype=torch.int32)
    dist.all_gather_into_tensor(out, x)
    torch.cuda.synchronize()
    print(f"rank {rank}: all_gather {out.tolist()}", flush=True)
    from vitparticlefiltertracker_amd.particle_filter import ParticleFilter
    P = 4096
    pfs = ParticleFilter(P, (100.0, 90.0, 1.0), rank=rank, world_size=world, seed=7)
    ref = ParticleFilter(P, (100.0, 90.0, 1.0), seed=7)
    g = torch.Generator(device="cuda").manual_seed(3)
    ok = True
    for k in range(1, 6):
        Q = torch.randint(0, 1 << 40, (P,), device="cuda", generator=g, dtype=torch.int64)
        if k == 2:
            Q.zero_()
        pfs.predict(k)
        ref.predict(k)
        pfs.set_weights(Q[rank * pfs.n_local:(rank + 1) * pfs.n_local])
        ref.set_weights(Q)
        e1, e0 = pfs.step(), ref.step()
        same = (e1 == e0 and torch.equal(pfs.last_ancestors, ref.last_ancestors[rank * pfs.n_local:(rank + 1) * pfs.n_local])
                and torch.equal(pfs.particles_soa, ref.particles_soa[:, rank * pfs.n_local:(rank + 1) * pfs.n_local]))
        ok &= same
        print(f"rank {rank} frame {k}: estimate {e1} single-rank {e0} bit-exact {same}", flush=True)
    dist.destroy_process_group()
    print(f"rank {rank}: RCCL PF exchange {'OK' if ok else 'MISMATCH'}", flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
