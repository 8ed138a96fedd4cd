"""GPU: one PGTrainer iteration (no Adam) at every BASELINE workload's full size
(workloads.py: C2 easy 4096x200, C3 default + CurriculumScheduler 4096x200, C4 hard
held-out table 8192x200, C5 variable + noise 0.05 4096x200), each checked three ways:

1. the learner: V / adv / ret / normalisation stats / every gradient block against
   tests/pg_reference.py run in torch fp32 on the device (bf16 storage points emulated);
2. GAE + advantage normalisation in isolation: the device's own V, rew and done fed to
   pg_reference.gae must give the kernel's adv / ret to 1e-5 (north star), and the
   one-pass f64 mean / std must equal a two-pass f64 reduction of the kernel's adv;
3. the rollout tape: >= 32 lanes (first, last, every 16-env workgroup boundary probed,
   random) replayed for all 200 steps by the CPU oracle -- the oracle's own noisy action /
   observation from the policy action and the noise values the kernel drew (config C5),
   auto-resets from the oracle's Philox restatement -- applied actions / rewards / dones /
   obs equal; the noise values themselves pinned to their Philox draws and moments.

Reference analogue: the returns of training/episode_utils.py:42-53 (the reference has no
GAE or network learner: parity of the learner itself is unpinned)."""
import math

import numpy as np
import pytest
import torch

import pg_reference as R
from oracle.dx_oracle import (STREAM_DYN, STREAM_OBS, OracleCurriculum, OracleEnv, device_normals_f64, env_key,
                              oracle_noisy_action, oracle_noisy_obs, philox_reset_draws)

pytestmark = pytest.mark.gpu
CONFIGS = ["easy", "default", "hard_heldout", "variable_noise"]


def env_key_np(seed, gid):
    k = [env_key(seed, int(g)) for g in gid]
    return np.array([a for a, _ in k], np.uint64), np.array([b for _, b in k], np.uint64)


@pytest.fixture(scope="module")
def pkg():
    import dexterous_rl_manipulation_amd as d
    from dexterous_rl_manipulation_amd import trainer, workloads  # noqa: F401
    return d


def _run(pkg, name, **kw):
    dev = torch.device("cuda", 0)
    env, tr = pkg.workloads.build_pg_workload(name, dev, ent_coef=0.01, **kw)
    tr.applied_act = torch.zeros(tr.M, 16, device=dev)
    tr.dyn_noise_tape = torch.full((tr.M, 16), float("nan"), device=dev)
    tr.obs_noise_tape = torch.full((tr.M + tr.n, 48), float("nan"), device=dev)
    st0 = {k: getattr(env, k).clone() for k in ("joint_positions", "object_position", "object_size", "object_mass",
                                                 "friction_coefficient", "curriculum_index", "reset_counter")}
    st0["curricula"] = list(env.curriculum_configs)  # C3: a progression swaps the table after the iteration
    for ph in tr.phases():
        if ph != "optimizer_step":
            getattr(tr, ph)()
    torch.cuda.synchronize()
    return env, tr, st0


def _oracle_cur(c):
    return OracleCurriculum(object_size=c.object_size, object_mass=c.object_mass,
                            friction_coefficient=c.friction_coefficient, size_range=c.object_size_range,
                            mass_range=c.object_mass_range, friction_range=c.friction_range,
                            spawn_x_range=c.spawn_x_range, spawn_y_range=c.spawn_y_range,
                            spawn_z_range=c.spawn_z_range,
                            friction_is_np_float64=bool(c.to_native().friction_is_f64_scalar))


def _lanes(n, k=32, seed=0):
    probe = [0, 1, 7, 8, 15, 16, 17, 31, 32, 63, 64, 255, 256, n // 2 - 1, n // 2, n - 33, n - 32, n - 17, n - 16,
             n - 1]
    rng = np.random.default_rng(seed)
    rest = rng.choice(np.setdiff1d(np.arange(n), probe), k - len(probe) + 4, replace=False)
    return sorted(set(probe) | set(int(x) for x in rest))


@pytest.fixture(scope="module", params=CONFIGS)
def run(request, pkg):
    return (request.param,) + _run(pkg, request.param)


def test_learner_matches_torch_reference(run):
    name, env, tr, _ = run
    n, T = tr.n, tr.T
    c = tr.cfg
    cfg = dict(gamma=c.gamma, lam=c.lam, clip_eps=c.clip_eps, vf_coef=c.vf_coef, ent_coef=c.ent_coef)
    g_ref, info = R.loss_and_grads(tr.params.clone(), tr.obs_rm, tr.act, tr.logp, tr.rew, tr.done, n, T, cfg,
                                   bf16=True)
    # bf16 ties: see test_gpu_pg.test_iteration_matches_torch_reference for the tolerances
    torch.testing.assert_close(tr.V[0], info["V"], rtol=1e-2, atol=3e-3)
    assert (tr.V[0] - info["V"]).norm() / info["V"].norm() < 2e-3
    torch.testing.assert_close(tr.adv, info["adv"], rtol=1e-2, atol=5e-3)
    torch.testing.assert_close(tr.ret, info["ret"], rtol=1e-2, atol=5e-3)
    assert math.isclose(tr.stats[4].item(), info["std"].item(), rel_tol=1e-3)
    T_ = __import__("dexterous_rl_manipulation_amd").trainer
    for blk in ("W1a", "W2a", "W3a", "W1c", "W2c", "W3c"):
        got, ref = tr.block(blk, tr.grads), R.unpack(g_ref)[blk]
        rel = (got - ref).norm() / ref.norm().clamp_min(1e-12)
        cos = torch.nn.functional.cosine_similarity(got.flatten(), ref.flatten(), dim=0)
        assert rel < 2e-2 and cos > 0.9998, (name, blk, rel.item(), cos.item())
    ls = slice(T_.OFF["logstd"], T_.OFF["logstd"] + 15)
    torch.testing.assert_close(tr.grads[ls], g_ref[ls], rtol=1e-3, atol=1e-6)
    ls_ = tr.loss_stats()
    assert ls_["clip_frac"] == 0.0 and abs(ls_["approx_kl"]) < 1e-9  # rollout policy == training forward
    # fp64 truth: no block, nor V / adv, further from it than 1.5 x the bf16 torch reference
    R.fp64_pin(tr.grads, tr.V[0], tr.adv, tr.params.clone(), tr.obs_rm, tr.act, tr.logp, tr.rew, tr.done, n, T, cfg,
               g_ref, info)


def test_gae_and_normalisation_isolated(run):
    name, env, tr, _ = run
    n, T = tr.n, tr.T
    adv, ret = R.gae(tr.rew, tr.done, tr.V[0], n, T, tr.cfg.gamma, tr.cfg.lam)
    torch.testing.assert_close(tr.adv, adv, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(tr.ret, ret, rtol=1e-5, atol=1e-6)
    a = tr.adv.double()
    assert tr.stats[0].item() == n * T
    assert math.isclose(tr.stats[2].item(), a.mean().item(), rel_tol=1e-9, abs_tol=1e-12)
    assert math.isclose(tr.stats[4].item(), a.std().item(), rel_tol=1e-9)


def test_rollout_tape_matches_oracle(run):
    """>= 32 lanes replayed by the oracle for all 200 steps.  The oracle steps with the action
    IT derives from the policy's tape action and the dynamics noise the kernel drew:
    clip(f32(a + f32(n)), -1, 1) (oracle_noisy_action, robustness_tests.py:177-187), which must
    equal the action the kernel integrated (applied_act) bit for bit; every observation row must
    equal bf16(f32(obs + f32(n_obs))) (oracle_noisy_obs, robustness_tests.py:199-207) with the
    observation noise the kernel drew.  Without noise the same check runs with n = 0."""
    name, env, tr, st0 = run
    n, T = tr.n, tr.T
    rew, done = tr.rew.view(T, n).cpu().numpy(), tr.done.view(T, n).cpu().numpy()
    applied = tr.applied_act.view(T, n, 16).cpu().numpy()
    pol_act = tr.act.view(T, n, 16).cpu().numpy()
    nd = tr.dyn_noise_tape.view(T, n, 16).cpu().numpy()
    no = tr.obs_noise_tape.view(T + 1, n, 48).cpu().numpy()
    obs = tr.obs_rm.view(T + 1, n, 64).float().cpu().numpy()
    s = {k: v.cpu().numpy() for k, v in st0.items() if k != "curricula"}
    curs = [_oracle_cur(c) for c in st0["curricula"]]
    seed = env._cfg.seed
    dyn_on, obs_on = tr.cfg.dyn_noise_std > 0, tr.cfg.obs_noise_std > 0
    if not dyn_on:
        assert not nd.any()
    lanes = _lanes(n)
    assert len(lanes) >= 32
    resets = 0
    bf = lambda x: torch.from_numpy(np.asarray(x, np.float32)).to(torch.bfloat16).float().numpy()  # noqa: E731

    def want_row(ob, t, i):
        return bf(oracle_noisy_obs(np.asarray(ob, np.float32), no[t, i, :45]) if obs_on else ob)

    for i in lanes:
        cur = curs[int(s["curriculum_index"][i])]
        orc = OracleEnv(cur=cur, dense=True, max_episode_steps=env.max_episode_steps)
        d = np.full(21, np.nan)
        d[:15] = s["joint_positions"][:, i]
        d[15:18] = s["object_size"][i], s["object_mass"][i], s["friction_coefficient"][i]
        d[18:21] = s["object_position"][:, i]
        ob = orc.reset(d)
        k0, k1 = env_key(seed, env._cfg.global_env_offset + i)
        ctr = int(s["reset_counter"][i]) & ((1 << 64) - 1)
        for t in range(T):
            assert np.array_equal(obs[t, i, :45], want_row(ob, t, i)), (name, i, t)
            a = pol_act[t, i, :15]
            if dyn_on:
                a = np.asarray(oracle_noisy_action(a, nd[t, i, :15]), np.float32)
            assert np.array_equal(applied[t, i, :15], a), (name, i, t)
            ob, r, te, trn = orc.step(a)
            r32 = np.float32(r)
            assert abs(rew[t, i] - r32) <= np.spacing(abs(r32)), (name, i, t, rew[t, i], r)
            d_ = te or trn or orc.t >= tr.max_steps
            assert bool(done[t, i]) == d_, (name, i, t)
            if d_:
                ob = orc.reset(philox_reset_draws(cur, k0, k1, ctr))
                ctr += 1
                resets += 1
        assert np.array_equal(obs[T, i, :45], want_row(ob, T, i)), (name, i, "bootstrap")
    assert resets > 0


def test_fused_noise_streams(run):
    """Config C5's noise as drawn: the dynamics / observation noise tapes hold f32(sigma) * z
    with z the Box-Muller normal of the lane's own Philox block (policy key of the global env
    id, counter iteration * T + t, the dyn / obs stream, block = element // 4) -- checked
    against the oracle's f64 restatement of those draws on the sampled lanes (hardware
    log / sqrt / sin / cos: ~1e-6 relative, so this pins WHICH draws were added, the exact
    arithmetic applied to them is test_rollout_tape_matches_oracle's) -- and their moments over
    the whole 4096 x 200 tape (mean 0, std sigma).  The reference draws n = N(0, sigma) in f64
    and rounds to f32 (robustness_tests.py:181-182, :203-204); the kernel rounds sigma to f32
    and multiplies in f32."""
    name, env, tr, _ = run
    c = tr.cfg
    if c.dyn_noise_std <= 0 and c.obs_noise_std <= 0:
        pytest.skip("no fused noise in this workload")
    n, T = tr.n, tr.T
    nd = tr.dyn_noise_tape.view(T, n, 16).double().cpu().numpy()
    no = tr.obs_noise_tape.view(T + 1, n, 48).double().cpu().numpy()
    assert not np.isnan(nd).any() and not np.isnan(no).any()
    assert not nd[:, :, 15:].any() and not no[:, :, 45:].any()
    pseed = (int(c.seed) * 0x9E3779B97F4A7C15 + 17) & (2**64 - 1)
    lanes = np.array(_lanes(n))
    gid = env._cfg.global_env_offset + lanes
    key = env_key_np(pseed, gid)
    for sig, tape, stream, blocks, rows, width in ((c.dyn_noise_std, nd, STREAM_DYN, 4, T, 15),
                                                   (c.obs_noise_std, no, STREAM_OBS, 12, T + 1, 45)):
        sig32 = float(np.float32(sig))
        vals = tape[:, :, :width]
        N_ = vals.size
        assert abs(vals.mean()) < 6 * sig / math.sqrt(N_), (name, vals.mean())
        assert abs(vals.std() / sig - 1.0) < 2e-3, (name, vals.std())
        # Kolmogorov-Smirnov distance of the whole tape (4096 x 200 x 15 / 4096 x 201 x 45 draws)
        # to N(0, sigma), on the device; 1.95 / sqrt(N) is the 0.1 % critical value.  The generator
        # (Philox2x32-10, 24-bit radius and 16-bit angle uniforms, |z| <= 5.77)
        # is the build's own: it carries distributional parity with the reference's
        # default_rng normals, not value parity
        x = torch.from_numpy(vals.reshape(-1)).to("cuda").sort().values / sig32
        cdf = torch.special.ndtr(x)
        k = torch.arange(1, x.numel() + 1, device=x.device, dtype=torch.float64) / x.numel()
        ks = torch.maximum(k - cdf, cdf - (k - 1.0 / x.numel())).max().item()
        assert ks < 1.95 / math.sqrt(N_), (name, stream, ks)
        # the tail (the 16-bit radius uniform of round 5 capped |z| at 4.71 and the
        # KS distance cannot see a missing 2.5e-6 of mass): P(|z| > 4) and P(|z| > 4.5) within 5
        # binomial sigma of the normal's, and draws beyond 4.71 sigma present
        a = x.abs()
        for thr, pt in ((4.0, 6.334248366623996e-05), (4.5, 6.795346249477e-06)):
            cnt, mu = (a > thr).sum().item(), pt * N_
            assert abs(cnt - mu) < 5 * math.sqrt(mu * (1 - pt)), (name, stream, thr, cnt, mu)
        assert a.max().item() > 4.72, (name, stream, a.max().item())
        ctr = (np.uint64(tr.iteration_index) * np.uint64(T) + np.arange(rows, dtype=np.uint64))[:, None]
        ctr = np.broadcast_to(ctr, (rows, len(lanes)))
        z = device_normals_f64((key[0][None, :], key[1][None, :]), ctr, stream, blocks)[..., :width]
        got = vals[:rows][:, lanes]
        err = np.abs(got - sig32 * z)
        assert (err <= sig32 * (1e-4 + 1e-4 * np.abs(z))).all(), (name, stream, err.max())


@pytest.mark.parametrize("name", CONFIGS)
def test_benched_rollout_equals_parity_instantiation(pkg, name):
    """The bench runs k_pg_rollout_ws<noise, kDiag=false>; the oracle tests above check
    <noise, true> (selected by the parity tapes).  From one snapshot of the env state slab and
    the open-episode returns, the rollout runs once with the tapes and once without: every
    tape (obs / act / log pi / rew / done / episode codes), the per-env sums, the episode
    records and the env state after the launch are bit-identical.  Second iteration: the
    state going in has mid-episode envs and the Philox counters have moved."""
    dev = torch.device("cuda", 0)
    env, tr = pkg.workloads.build_pg_workload(name, dev, record_cap=8)
    tr.rollout()  # advance into mid-episode state
    tr.iteration_index += 1
    if tr.ep_code is None:
        tr.ep_code = torch.zeros(tr.M, dtype=torch.int16, device=dev)
    torch.cuda.synchronize()
    snap, ret0 = env.state.clone(), tr.ep_ret.clone()
    outs = []
    for tapes in (True, False):
        env.state.copy_(snap)
        tr.ep_ret.copy_(ret0)
        for t in (tr.obs_rm, tr.act, tr.logp, tr.rew, tr.done, tr.ep_count, tr.ep_sum_ret, tr.ep_sum_len, tr.ep_succ,
                  tr.rec_return, tr.rec_length, tr.rec_success, tr.rec_end, tr.ep_code):
            t.fill_(0x5A if t.dtype in (torch.uint8,) else 7)
        tr.applied_act = torch.zeros(tr.M, 16, device=dev) if tapes else None
        tr.dyn_noise_tape = torch.zeros(tr.M, 16, device=dev) if tapes else None
        tr.obs_noise_tape = torch.zeros(tr.M + tr.n, 48, device=dev) if tapes else None
        tr.rollout()
        torch.cuda.synchronize()
        outs.append({k: getattr(tr, k).clone() for k in (
            "obs_rm", "act", "logp", "rew", "done", "ep_count", "ep_sum_ret", "ep_sum_len", "ep_succ", "rec_return",
            "rec_length", "rec_success", "rec_end", "ep_code", "ep_ret")} | {"state": env.state.clone()})
    a, b = outs
    for k in a:
        assert a[k].view(torch.uint8).equal(b[k].view(torch.uint8)), (name, k)
    assert int(a["ep_count"].sum()) > 0


_STATE_FIELDS = ("joint_positions", "joint_velocities", "object_position", "object_velocity", "flags", "step_count",
                 "object_size", "object_mass", "friction_coefficient", "curriculum_index", "reset_counter")


@pytest.mark.parametrize("name", ["hard_heldout", "variable_noise"])
def test_32_env_kernel_equals_16_env_kernel_at_full_size(pkg, name):
    """At C4's 8192 envs (32 per CU) the rollout runs k_pg_rollout_e8 (8 lanes per env, 32 envs
    per workgroup, one round); the 16-env k_pg_rollout_ws (diag 2048) must give the same tapes,
    per-env sums, records and env state bit for bit, over two iterations (mid-episode state and
    moved Philox counters in the second).  variable_noise at 8192 envs runs the e8 kernel's
    fused observation / dynamics noise."""
    dev = torch.device("cuda", 0)
    outs = []
    for diag in (0, 2048):
        env, tr = pkg.workloads.build_pg_workload(name, dev, envs=8192, record_cap=8)
        if tr.ep_code is None:
            tr.ep_code = torch.zeros(tr.M, dtype=torch.int16, device=dev)
        tr.diag_flags = diag
        for _ in range(2):
            tr.rollout()
            tr.iteration_index += 1
        torch.cuda.synchronize()
        outs.append({k: getattr(tr, k).clone() for k in (
            "obs_rm", "act", "logp", "rew", "done", "ep_count", "ep_sum_ret", "ep_sum_len", "ep_succ", "rec_return",
            "rec_length", "rec_success", "rec_end", "ep_code", "ep_ret")}
                    | {k: getattr(env, k).clone() for k in _STATE_FIELDS})  # the fields, not the slab's padding
        del env, tr
    a, b = outs
    for k in a:
        assert a[k].view(torch.uint8).equal(b[k].view(torch.uint8)), (name, k)
    assert int(a["ep_count"].sum()) > 0


def test_normalisation_large_mean(pkg):
    """The normalisation moments with |mean| / std > 1e3 (every step its own episode,
    A = r - V, rewards shifted by 1e4): a one-pass sum(a^2) - mean sum(a) lost 2.8e-6 of
    the std here; the merged (count, mean, M2) moments (k_gae / k_gae_sums /
    k_stats_combine) match a two-pass f64 reduction of the kernel's advantages to 1e-9."""
    dev = torch.device("cuda", 0)
    env, tr = pkg.workloads.build_pg_workload("easy", dev)
    tr.rollout()
    tr.critic_values()
    tr.rew.add_(1e4)
    tr.done.fill_(1)
    tr.advantages()
    torch.cuda.synchronize()
    a = tr.adv.double()
    ratio = abs(a.mean().item()) / a.std().item()
    assert ratio > 1e3, ratio
    assert math.isclose(tr.stats[2].item(), a.mean().item(), rel_tol=1e-12)
    assert math.isclose(tr.stats[4].item(), a.std().item(), rel_tol=1e-9)
