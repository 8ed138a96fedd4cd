"""CPU: the manual PG backward (pg_reference.py, mirrored by the HIP kernels)
equals torch autograd on the same PPO + value + entropy objective (fp64)."""
import pytest
import torch

import pg_reference as R


def make_case(n=8, T=6, seed=0, dtype=torch.float64):
    g = torch.Generator().manual_seed(seed)
    params = torch.zeros(R.NPARAMS, dtype=dtype)
    Wd = R.unpack(params)
    for net in "ac":
        Wd[f"W1{net}"][:, :R.OBS_IN + 1] = 0.2 * torch.randn(R.H, R.OBS_IN + 1, generator=g, dtype=dtype)
        Wd[f"W2{net}"][:, :R.H + 1] = 0.08 * torch.randn(R.H, R.H + 1, generator=g, dtype=dtype)
        rows = R.ACT if net == "a" else 1
        Wd[f"W3{net}"][:rows, :R.H + 1] = 0.1 * torch.randn(rows, R.H + 1, generator=g, dtype=dtype)
    Wd["logstd"][:] = -0.5 + 0.1 * torch.randn(R.ACT, generator=g, dtype=dtype)
    obs = torch.zeros((T + 1) * n, R.IN, dtype=dtype)
    obs[:, :R.OBS_IN] = torch.randn((T + 1) * n, R.OBS_IN, generator=g, dtype=dtype)
    obs[:, R.OBS_IN] = 1.0
    M = n * T
    act = torch.zeros(M, 16, dtype=dtype)
    act[:, :R.ACT] = torch.randn(M, R.ACT, generator=g, dtype=dtype)
    rew = torch.rand(M, generator=g, dtype=dtype)
    done = (torch.rand(M, generator=g) < 0.15).to(torch.uint8)
    with torch.no_grad():
        _, _, mh = R.mlp_forward(obs[:M], R.unpack(params), "a", False)
        mu, ls = mh[:, :R.ACT], R.unpack(params)["logstd"]
        lp = (-0.5 * ((act[:, :R.ACT] - mu) * torch.exp(-ls)) ** 2 - ls - 0.5 * R.LOG2PI).sum(1)
    logp_old = lp + 0.3 * torch.randn(M, generator=g, dtype=dtype)  # ratios != 1: clipping active
    return params, obs, act, logp_old, rew, done


CFG = dict(gamma=0.99, lam=0.95, clip_eps=0.2, vf_coef=0.5, ent_coef=0.01)


def test_manual_backward_matches_autograd():
    n, T = 8, 6
    params, obs, act, logp_old, rew, done = make_case(n, T)
    grads, info = R.loss_and_grads(params, obs, act, logp_old, rew, done, n, T, CFG, bf16=False)
    ref = R.autograd_loss(params, obs, act, logp_old, rew, done, n, T, CFG)
    assert ((info["ratio"] - 1).abs() > CFG["clip_eps"]).any()  # the clipped branch is exercised
    torch.testing.assert_close(grads, ref, rtol=1e-9, atol=1e-12)


def test_gae_matches_closed_form_single_episode():
    n, T, gamma, lam = 1, 5, 0.9, 0.8
    rew = torch.arange(1, T + 1, dtype=torch.float64)
    done = torch.zeros(T, dtype=torch.uint8)
    V = torch.linspace(0.5, 1.5, T + 1, dtype=torch.float64)
    adv, ret = R.gae(rew, done, V, n, T, gamma, lam)
    deltas = rew + gamma * V[1:] - V[:-1]
    expect = torch.tensor([sum((gamma * lam) ** (k - t) * deltas[k] for k in range(t, T)) for t in range(T)],
                          dtype=torch.float64)
    torch.testing.assert_close(adv, expect)
    torch.testing.assert_close(ret, expect + V[:-1])
    done[2] = 1  # episode boundary cuts the bootstrap and the trace
    adv2, _ = R.gae(rew, done, V, n, T, gamma, lam)
    assert abs(adv2[2] - (rew[2] - V[2])) < 1e-12


@pytest.mark.parametrize("n,T,p_done", [(7, 1, 0.0), (5, 9, 0.2), (33, 200, 0.02), (4, 129, 0.0), (3, 600, 0.05)])
def test_gae_segmented_scan_equals_sequential_recurrence(n, T, p_done):
    """k_gae_lds's segmented scan (restated op for op by pg_reference.gae) against the one-chain
    f32 recurrence and an f64 one: the composition only re-rounds each segment's incoming value, so
    the two f32 forms agree to a few ulp of the chain's magnitude and both sit within 1e-5 of f64
    (north star: returns within 1e-5)."""
    g = torch.Generator().manual_seed(1000 * n + T)
    rew = torch.randn(T * n, generator=g)
    V = torch.randn((T + 1) * n, generator=g) * 3.0
    done = (torch.rand(T * n, generator=g) < p_done).to(torch.uint8)
    a_scan, r_scan = R.gae(rew, done, V, n, T, 0.99, 0.95, scan=True)
    a_seq, r_seq = R.gae(rew, done, V, n, T, 0.99, 0.95, scan=False)
    a64, _ = R.gae(rew.double(), done, V.double(), n, T, 0.99, 0.95, scan=False)
    scale = a64.abs().max().item() + 1.0
    assert (a_scan.double() - a_seq.double()).abs().max().item() <= 1e-6 * scale
    assert (a_scan.double() - a64).abs().max().item() <= 1e-5 * scale
    torch.testing.assert_close(r_scan, a_scan + V.view(T + 1, n)[:T].reshape(-1), rtol=0, atol=0)
    if T <= 8:  # one chunk: a single segment holds the whole horizon, no composition at all
        assert torch.equal(a_scan, a_seq)


def test_fp64_pin_ratios():
    """pg_reference.fp64_pin: the bf16-emulating reference itself sits at ratio 1 of its own
    distance to the fp64 truth; a result with doubled error (got = truth + 2 (ref - truth))
    is rejected."""
    import pytest
    n, T = 8, 6
    params, obs, act, logp_old, rew, done = make_case(n, T, dtype=torch.float32)
    logp_old = logp_old.float()
    g, info = R.loss_and_grads(params, obs, act, logp_old, rew, done, n, T, CFG, bf16=True)
    r = R.fp64_pin(g, info["V"], info["adv"], params, obs, act, logp_old, rew, done, n, T, CFG, g, info)
    assert all(abs(v - 1.0) < 1e-6 for v in r.values()), r
    g64, info64 = R.loss_and_grads(params.double(), obs, act, logp_old, rew, done, n, T, CFG, bf16=False)
    worse = g.double() + (g.double() - g64)
    with pytest.raises(AssertionError):
        R.fp64_pin(worse, info["V"], info["adv"], params, obs, act, logp_old, rew, done, n, T, CFG, g, info)
