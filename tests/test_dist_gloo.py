"""CPU, world_size 2, 3 and 8 over gloo: the sharded learner decomposition equals the
single-process learner on the concatenated batch.

Each rank takes its shard of the envs (distributed.shard_range), runs the same
per-shard math the HIP pipeline runs (pg_reference, fp64) and exchanges exactly
what PGTrainer exchanges, through the functions PGTrainer itself calls
(dexterous_rl_manipulation_amd.distributed):
  * the local advantage moments in the trainer's f64[8] stats layout (count, mean,
    sum of squared deviations at [5..7]) -> gather_adv_moments_ (one all-gather)
    -> combine_adv_moments (rank-order Chan merge, the restatement of csrc
    k_stats_combine);
  * global_count + loss_scales -> the per-sample 1/(global samples) scale and the
    per-rank ent_coef/world the kernels receive (ragged shards included);
  * the SUM all-reduce of the flat gradient buffer, also in the trainer's two-halves form
    (the critic half overlapped with the actor's train pass) == one all-reduce.
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
    n, T = 9, 6  # 9 envs: ragged shards for world 2 (4 + 5) and 8 (2 + 7 x 1), even ones for world 3
    params, obs, act, logp_old, rew, done = make_case(n, T, seed=3)
    full, full_info = R.loss_and_grads(params, obs, act, logp_old, rew, done, n, T, CFG, bf16=False)
    lo, hi = D.shard_range(n, world, rank)
    nl = hi - lo
    o = _shard(obs, T + 1, n, lo, hi)
    a, lp, rw, dn = (_shard(x, T, n, lo, hi) for x in (act, logp_old, rew, done))

    seen = {}

    def norm_stats(adv):
        stats = torch.zeros(8, dtype=torch.float64)  # PGTrainer.stats as dxrl_pg_gae leaves it
        a64 = adv.double()
        stats[5], stats[6], stats[7] = float(adv.numel()), a64.mean(), ((a64 - a64.mean()) ** 2).sum()
        stats[2] = 123.0  # a stale mean from a previous iteration must not leak into the exchange
        out = torch.zeros(topo.world, 3, dtype=torch.float64)
        D.gather_adv_moments_(out, stats, topo.world, topo.group)
        n_, mean, m2, std = D.combine_adv_moments(out)
        seen["moments"] = (n_, n_ * mean)
        return torch.tensor(mean, dtype=torch.float64), torch.tensor(std, dtype=torch.float64)

    scales = D.loss_scales(D.global_count(nl * T, topo.world, topo.group), world, CFG["ent_coef"])
    g, info = R.loss_and_grads(params, o, a, lp, rw, dn, nl, T, CFG, bf16=False, norm_stats=norm_stats,
                               scales=scales)
    # the trainer's overlapped form: the critic half (the tail of the buffer) reduced on its own,
    # then the actor half -- element-wise the same SUM as one all-reduce of the whole buffer
    gs = g.clone()
    cut = gs.numel() // 3
    D.all_reduce_sum_(gs[cut:], topo.world, topo.group)
    D.all_reduce_sum_(gs[:cut], topo.world, topo.group)
    D.all_reduce_sum_(g, topo.world, topo.group)
    if world == 2:
        assert torch.equal(gs, g)  # a + b: no order to differ in
    else:
        assert torch.allclose(gs, g, rtol=1e-12, atol=1e-15)
    # the global moments are those of the concatenated batch
    adv_full = full_info["adv"].double()
    assert seen["moments"][0] == n * T
    assert abs(seen["moments"][1] - adv_full.sum().item()) < 1e-9 * adv_full.abs().sum().item()
    assert abs(info["std"].item() - adv_full.std().item()) < 1e-9 * adv_full.std().item()
    # the scheduler feed's all-gather of u16 episode-end codes (moved as bytes), rank-major
    codes = (torch.arange(12, dtype=torch.int32) * 1000 + rank * 7 + 40000).to(torch.int16)
    allc = torch.zeros(world * 12, dtype=torch.int16)
    D.all_gather_into_(allc, codes, topo.world, topo.group)
    for r in range(world):
        assert torch.equal(allc[r * 12:(r + 1) * 12], (torch.arange(12, dtype=torch.int32) * 1000 + r * 7 + 40000)
                           .to(torch.int16))
    err = (g - full).abs().max().item()
    scale = full.abs().max().item()
    out[rank] = err / scale
    import torch.distributed as dist
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_gloo_exchange_equals_concatenated_batch(world):
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    assert len(out) == world and max(out.values()) < 1e-9, dict(out)


@pytest.mark.parametrize("n,world", [(8, 2), (4096, 8), (10, 3), (7, 4)])
def test_shard_ranges_partition(n, world):
    from dexterous_rl_manipulation_amd.distributed import shard_range
    spans = [shard_range(n, world, r) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    assert all(spans[k][1] == spans[k + 1][0] for k in range(world - 1))
    assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1
