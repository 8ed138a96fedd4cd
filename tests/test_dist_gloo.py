"""CPU, world_size 2 over gloo: the sharded learner decomposition equals the
single-process learner on the concatenated batch.

Each rank takes half of the envs, runs the same per-shard math the HIP
pipeline runs (pg_reference, fp64), and exchanges exactly what PGTrainer
exchanges through dexterous_rl_manipulation_amd.distributed: (count, sum)
and the squared-deviation sum of the advantages (global two-pass
normalisation), then one SUM all-reduce of the flat gradient buffer.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

import pg_reference as R
from test_pg_reference import CFG, make_case


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _shard(t, T1, n, lo, hi):
    return t.view(T1, n, *t.shape[1:])[:, lo:hi].reshape(-1, *t.shape[1:])


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import dexterous_rl_manipulation_amd  # noqa: F401
    from dexterous_rl_manipulation_amd import distributed as D
    topo = D.init_from_env(backend="gloo")
    n, T = 8, 6
    params, obs, act, logp_old, rew, done = make_case(n, T, seed=3)
    full, _ = R.loss_and_grads(params, obs, act, logp_old, rew, done, n, T, CFG, bf16=False)
    lo, hi = D.shard_range(n, world, rank)
    nl = hi - lo
    o = _shard(obs, T + 1, n, lo, hi)
    a, lp, rw, dn = (_shard(x, T, n, lo, hi) for x in (act, logp_old, rew, done))

    def norm_stats(adv):
        s = torch.tensor([float(adv.numel()), adv.double().sum().item()], dtype=torch.float64)
        D.all_reduce_sum_(s, topo.world, topo.group)
        mean = s[1] / s[0]
        q = torch.tensor([((adv.double() - mean) ** 2).sum().item()], dtype=torch.float64)
        D.all_reduce_sum_(q, topo.world, topo.group)
        return mean, torch.sqrt(q[0] / (s[0] - 1))

    g, _ = R.loss_and_grads(params, o, a, lp, rw, dn, nl, T, CFG, bf16=False, norm_stats=norm_stats,
                            total=n * T, world=world)
    D.all_reduce_sum_(g, topo.world, topo.group)
    err = (g - full).abs().max().item()
    scale = full.abs().max().item()
    out[rank] = err / scale
    import torch.distributed as dist
    dist.destroy_process_group()


def test_world2_gloo_equals_concatenated_batch():
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    assert len(out) == 2 and max(out.values()) < 1e-9, dict(out)


@pytest.mark.parametrize("n,world", [(8, 2), (4096, 8), (10, 3), (7, 4)])
def test_shard_ranges_partition(n, world):
    from dexterous_rl_manipulation_amd.distributed import shard_range
    spans = [shard_range(n, world, r) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    assert all(spans[k][1] == spans[k + 1][0] for k in range(world - 1))
    assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1
