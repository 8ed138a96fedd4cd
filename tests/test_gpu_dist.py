"""GPU, multi-rank: PGTrainer sharded over two and four ranks (processes on cuda:0, gloo
process group -- RCCL needs one GPU per rank, which a one-GPU test box does not
have) equals the world-1 trainer on the concatenated batch ("the
8-rank loss/params must equal 1-rank on the concatenated batch within fp32
reduction-order tolerance").  Same global env ids -> bit-identical rollout tapes;
the gradient SUM and the advantage moments differ from world 1 only in
summation order."""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(tmp, world, n, iters, config, mode="0"):
    """mode: "0" the default trainer (serialised exchanges, paired learner step), "1" exchanges on
    the side stream, "u" serialised with one learner call per network."""
    port = _port()
    procs, outs = [], []
    for r in range(world):
        out = os.path.join(tmp, f"w{world}_r{r}_m{mode}.pt")
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_pg_worker.py"), out, str(n),
                                       str(iters), config, mode], env=env))
        outs.append(out)
    for p in procs:
        assert p.wait(timeout=240) == 0
    return [torch.load(o, weights_only=False) for o in outs]


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("config", ["variable", "default"])
def test_ranks_equal_one_rank_on_concatenated_batch(tmp_path, config, world):
    """world ranks of n envs == one rank of world x n envs (512 global envs either way; world 4
    drives the trainer's rank-order logic -- the moment merge, the C3 pack walk in (end step,
    global env id) order and the candidate-step all-reduce -- past two ranks)."""
    n, iters = 512 // world, 3
    one = _launch(str(tmp_path), 1, world * n, iters, config)[0]
    many = _launch(str(tmp_path), world, n, iters, config)
    # the first iteration's tapes: rank r holds env columns [r n, (r+1) n) of the world-1 run
    for r, res in enumerate(many):
        assert torch.equal(res["rew0"], one["rew0"][:, r * n:(r + 1) * n])
        assert torch.equal(res["done0"], one["done0"][:, r * n:(r + 1) * n])
    # every rank ends with the same parameters (identical Adam inputs after the all-reduce)
    for r in range(1, world):
        assert torch.equal(many[0]["params"], many[r]["params"]), r
        assert torch.equal(many[0]["stats0"][:5], many[r]["stats0"][:5]), r  # [5..7]: the rank's own moments
    # global advantage moments and normalisation == world 1 (f64, summation order only)
    for k in (0, 1, 2, 4):
        a, b = many[0]["stats0"][k].item(), one["stats0"][k].item()
        assert abs(a - b) <= 1e-9 * max(1.0, abs(b)), (k, a, b)
    # the first iteration's all-reduced gradient == the world-1 gradient (f32 summation order)
    gw, g1 = many[0]["grads0"], one["grads0"]
    rel = (gw - g1).norm() / g1.norm()
    assert rel < 1e-4, rel.item()
    # after `iters` Adam steps the parameters still agree to f32 reduction-order tolerance
    pw, p1 = many[0]["params"], one["params"]
    assert (pw - p1).abs().max().item() < 1e-4 * max(1.0, p1.abs().max().item())
    if config == "default":
        assert all(res["sched"] == one["sched"] for res in many)


@pytest.mark.parametrize("config", ["variable", "default"])
def test_overlapped_exchanges_equal_serialised(tmp_path, config):
    """Two ranks with the exchanges on the side stream (moment all-gather beside the critic's
    pass, the critic half of the gradient all-reduce beside the actor's, the scheduler codes
    beside critic values) == the same two ranks with every exchange serialised on the compute
    stream and the same per-network learner calls, bit for bit: the SUMs are element-wise the
    same (a + b at world 2)."""
    n, iters = 256, 3
    a = _launch(str(tmp_path), 2, n, iters, config, mode="1")
    b = _launch(str(tmp_path), 2, n, iters, config, mode="u")
    for r in range(2):
        for k in ("params", "grads0", "rew0", "done0", "stats0"):
            assert torch.equal(a[r][k], b[r][k]), (r, k)
        if config == "default":
            assert a[r]["sched"] == b[r]["sched"]
