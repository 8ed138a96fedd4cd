"""One process per GPU over torch.distributed (backend "nccl" = RCCL on ROCm).

The env side shards with no exchange: rank r owns global env ids
[r*N, (r+1)*N); every device RNG stream is keyed by the global id, so a
sharded run draws exactly what the same envs draw unsharded.  The PG learner
(trainer.PGTrainer) has two exchanges per iteration:
  * an all-gather of each rank's advantage moments (count, mean, sum of squared
    deviations; f64[3], contiguous at stats[5..7]), merged on every rank in rank
    order with Chan et al.'s pairwise update (csrc k_stats_combine, restated by
    ``combine_adv_moments``) -> the global normalisation, identical on all ranks;
  * one SUM all-reduce of the flat f32 gradient buffer.  The per-sample loss scale is 1/(global
    sample count) -- 1/(M*world) for equal shards -- and the entropy bonus
    enters each rank as ent_coef/world (``loss_scales``), so the SUM is the
    gradient of the global-batch mean loss (that algebra alone would also hold for
    ragged shards; the trainer requires equal ones, see below).
The curriculum scheduler (config C3) additionally all-gathers each rank's
episode-end codes so every rank feeds the same global episode stream.

Every helper runs its collective when ``world > 1`` OR a process group is passed:
a world-1 process group (``bench.py --dist``, tests/test_gpu_rccl.py) executes the
same RCCL calls a multi-rank job makes, whose results then equal their inputs.
Per-rank shards must be equal in size (the all-gathers and the scheduler's
global env ids assume it; PGTrainer checks).
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


def _active(world: int, group) -> bool:
    """Run the collective: several ranks, or an explicit process group (even of one rank)."""
    return world > 1 or group is not None


def _staged(t: torch.Tensor, group) -> bool:
    """gloo process groups (CPU tests, two ranks sharing one test GPU) exchange host copies."""
    import torch.distributed as dist
    return t.is_cuda and dist.get_backend(group) == "gloo"


def all_reduce_sum_(t: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """In-place SUM over ranks (no-op for world == 1 without a process group)."""
    if _active(world, group):
        import torch.distributed as dist
        if _staged(t, group):
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def all_gather_into_(out: torch.Tensor, t: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """out[r * t.numel():(r + 1) * t.numel()] = rank r's t (one collective; rank-major)."""
    if not _active(world, group):
        if out.data_ptr() != t.data_ptr():
            out.view(-1).copy_(t.view(-1))
        return out
    import torch.distributed as dist
    if t.dtype == torch.int16:  # neither RCCL nor gloo reduce 16-bit integers: move the bytes
        all_gather_into_(out.view(torch.uint8), t.contiguous().view(torch.uint8), world, group)
        return out
    if _staged(t, group):
        parts = [torch.empty_like(t, device="cpu") for _ in range(world)]
        dist.all_gather(parts, t.cpu(), group=group)
        out.view(world, -1).copy_(torch.stack([p.view(-1) for p in parts]))
    else:
        dist.all_gather_into_tensor(out.view(-1), t.view(-1), group=group)
    return out


def gather_adv_moments_(out: torch.Tensor, stats: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """out [world][3] = every rank's (count, mean, M2) block stats[5:8], in rank order
    (stats is the trainer's f64[8] vector as dxrl_pg_gae left it)."""
    return all_gather_into_(out, stats[5:8].contiguous(), world, group)


def merge_moments(a, b):
    """Chan, Golub & LeVeque's pairwise update of (count, mean, M2) (csrc/dxrl_pg.hip merge)."""
    if b[0] == 0.0:
        return a
    if a[0] == 0.0:
        return b
    n = a[0] + b[0]
    d = b[1] - a[1]
    return (n, a[1] + d * (b[0] / n), a[2] + b[2] + d * d * (a[0] * b[0] / n))


def combine_adv_moments(moments) -> tuple:
    """(count, mean, M2, unbiased std) from the ranks' triples merged in rank order -- exactly
    csrc k_stats_combine."""
    acc = (0.0, 0.0, 0.0)
    for row in moments:
        acc = merge_moments(acc, tuple(float(x) for x in row))
    n, mean, m2 = acc
    return n, mean, m2, (m2 / (n - 1.0 if n > 1.0 else 1.0)) ** 0.5


def loss_scales(global_samples: int, world: int, ent_coef: float) -> tuple:
    """(per-sample loss scale, per-rank entropy coefficient) of the sharded learner: each rank
    scales its samples by 1/(samples of all ranks) and adds ent_coef/world (the entropy term
    depends on the parameters only), so the SUM all-reduce of the rank gradients is the
    gradient of the mean loss over the concatenated batch."""
    return 1.0 / global_samples, ent_coef / world


def global_count(local: int, world: int, group=None) -> int:
    """SUM of a per-rank integer (one-time, at trainer construction)."""
    if not _active(world, group):
        return int(local)
    t = torch.tensor([int(local)], dtype=torch.int64)
    import torch.distributed as dist
    if dist.get_backend(group) == "nccl":
        t = t.cuda()
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return int(t.item())


def all_reduce_max(x: float, world: int, device, group=None) -> float:
    if not _active(world, group):
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def barrier(world: int, group=None):
    if _active(world, group):
        import torch.distributed as dist
        dist.barrier(group=group)


def shard_range(num_envs_global: int, world: int, rank: int):
    """Contiguous env shard of a rank (equal shards; the remainder goes to the last ranks)."""
    base, rem = divmod(num_envs_global, world)
    lo = rank * base + max(0, rank - (world - rem))
    return lo, lo + base + (1 if rank >= world - rem and rem else 0)
