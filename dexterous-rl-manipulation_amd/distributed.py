"""One process per GPU over torch.distributed (backend "nccl" = RCCL on ROCm).

The env side shards with no exchange: rank r owns global env ids
[r*N, (r+1)*N); every device RNG stream is keyed by the global id, so a
sharded run draws exactly what the same envs draw unsharded.  The PG learner
has three exchanges per iteration, all SUM all-reduces:
  * (count, sum) of the advantages, then the sum of squared deviations
    -> global two-pass normalisation;
  * one flat f32 gradient buffer (per-sample scale 1/(M*world), so the sum is
    the gradient of the global-batch mean loss).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch


@dataclass
class Topology:
    world: int
    rank: int
    local_rank: int
    device: torch.device
    group: Optional[object] = None

    @property
    def is_distributed(self) -> bool:
        return self.world > 1


def init_from_env(backend: Optional[str] = None) -> Topology:
    """Read RANK/LOCAL_RANK/WORLD_SIZE (torchrun) and join the process group.
    backend defaults to nccl (RCCL) with GPUs, gloo otherwise (CPU tests)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = torch.cuda.is_available()
    dev = torch.device("cuda", local) if gpu else torch.device("cpu")
    if gpu:
        torch.cuda.set_device(dev)
    group = None
    if world > 1:
        import torch.distributed as dist
        if not dist.is_initialized():
            be = backend or ("nccl" if gpu else "gloo")
            kw = {"device_id": dev} if be == "nccl" else {}
            dist.init_process_group(be, **kw)
        group = dist.group.WORLD
    return Topology(world, rank, local, dev, group)


def all_reduce_sum_(t: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """In-place SUM over ranks (no-op for world == 1)."""
    if world > 1:
        import torch.distributed as dist
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def all_reduce_max(x: float, world: int, device, group=None) -> float:
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def barrier(world: int, group=None):
    if world > 1:
        import torch.distributed as dist
        dist.barrier(group=group)


def shard_range(num_envs_global: int, world: int, rank: int):
    """Contiguous env shard of a rank (equal shards; the remainder goes to the last ranks)."""
    base, rem = divmod(num_envs_global, world)
    lo = rank * base + max(0, rank - (world - rem))
    return lo, lo + base + (1 if rank >= world - rem and rem else 0)
