"""GPU parity: the HIP path (through the C ABI) against the reference's golden
traces and the pinned CPU oracle.  Bit-exact for observations, flags, contact
counts, object position and learner state; rewards/returns within 1e-12 rel
(the north-star bar is 1e-5; f64 exp differs from numpy's by <= 1 ulp)."""
import math

import numpy as np
import pytest
import torch

import golden_io as G
from oracle.dx_oracle import OracleCurriculum, OracleEnv, reset_draws

pytestmark = pytest.mark.gpu

REW_RTOL = 1e-12


@pytest.fixture(scope="module")
def pkg():
    import dexterous_rl_manipulation_amd as d
    from dexterous_rl_manipulation_amd import envs, policies, training, experiments, evaluation  # noqa: F401
    assert torch.cuda.is_available()
    return d


def _pcg(seed):
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))


def _curriculum(pkg, rec):
    C = pkg.experiments.CurriculumConfig
    kw = {k: (tuple(v) if isinstance(v, list) else v) for k, v in rec.items() if not k.startswith("_")}
    c = C(**kw)
    for k in rec.get("_float64_scalars", []):
        setattr(c, k, np.float64(getattr(c, k)))
    return c


ENV_CASES = G.meta()["env_cases"]


@pytest.mark.parametrize("case", ENV_CASES, ids=lambda c: f"c{c['index']}-{c['cfg']}-{c['reward']}")
def test_facade_matches_reference_trace(pkg, case):
    """DexterousManipulationEnv facade: reset(seed)/step(action) == reference."""
    z = G.env_case(case["index"])
    env = pkg.envs.DexterousManipulationEnv(
        reward_type=case["reward"], curriculum_config=_curriculum(pkg, case["curriculum"]),
        max_episode_steps=case["max_episode_steps"],
        object_position=None if case.get("object_position") is None else np.array(case["object_position"]))
    for e in range(case["E"]):
        obs, info = env.reset(seed=case["seed"] if e == 0 else None)
        assert np.array_equal(obs, z["reset_obs"][e])
        assert np.array_equal(np.asarray(info["object_position"], np.float64), z["reset_op"][e])
        assert info["num_contacts"] == z["reset_ncon"][e]
        assert ("reward_components" in info) == bool(z["reset_has_comps"][e])
        for t in range(z["length"][e]):
            obs, r, term, trunc, info = env.step(z["actions"][e, t])
            assert np.array_equal(obs, z["obs"][e, t]), (e, t, np.flatnonzero(obs != z["obs"][e, t]))
            assert math.isclose(r, z["reward"][e, t], rel_tol=REW_RTOL, abs_tol=1e-15), (e, t)
            rc = info["reward_components"]
            np.testing.assert_allclose([rc["distance"], rc["contact"], rc["closure"], rc["stability"]],
                                       z["comps"][e, t], rtol=REW_RTOL, atol=1e-15)
            assert (term, trunc) == (bool(z["term"][e, t]), bool(z["trunc"][e, t]))
            assert info["num_contacts"] == z["ncon"][e, t]
            assert np.array_equal(info["object_position"], z["op"][e, t])
            assert info["step_count"] == z["step_count"][e, t]
    env.close()


def test_vecenv_batched_cases(pkg):
    """All dense/mes=200 trace episodes as lanes of ONE VecEnv (ragged N, per-env
    curriculum rows, masked resets): checks env indexing, LDS staging, tails."""
    cases = [c for c in ENV_CASES if c["reward"] == "dense" and c["max_episode_steps"] == 200
             and c.get("object_position") is None]
    lanes = []  # (case, episode) -- every episode of every case runs on its own lane
    for c in cases:
        for e in range(c["E"]):
            lanes.append((c, e))
    reps = 3  # replicate lanes so N is > 256 and not a multiple of 256
    lanes = lanes * reps
    n = len(lanes)
    assert n % 256 != 0
    cfgs = [_curriculum(pkg, c["curriculum"]) for c in cases]
    cidx = {id(c): k for k, c in enumerate(cases)}
    env = pkg.envs.VecEnv(n, reward_type="dense")
    env.set_curricula(cfgs, env_index=np.array([cidx[id(c)] for c, _ in lanes], np.int32))
    # every lane replays its case's whole trace (all episodes, sticky object included); per lane: sequence of (is_reset, draws | action) over its case's full trace
    seqs = []
    for c, _ in lanes:
        z = G.env_case(c["index"])
        ops = []
        for e in range(c["E"]):
            ops.append(("reset", z["draws"][e], z["reset_obs"][e], e))
            for t in range(z["length"][e]):
                ops.append(("step", z["actions"][e, t], (z["obs"][e, t], z["reward"][e, t], z["term"][e, t],
                                                         z["trunc"][e, t]), e))
        seqs.append(ops)
    dev = env.device
    for k in range(max(len(s) for s in seqs)):
        resets = [i for i, s in enumerate(seqs) if k < len(s) and s[k][0] == "reset"]
        steps = [i for i, s in enumerate(seqs) if k < len(s) and s[k][0] == "step"]
        if resets:
            mask = torch.zeros(n, dtype=torch.uint8)
            draws = torch.zeros(n, 21, dtype=torch.float64)
            for i in resets:
                mask[i] = 1
                draws[i] = torch.from_numpy(seqs[i][k][1])
            obs = env.reset(mask=mask.to(dev), draws=draws.to(dev)).cpu().numpy()
            for i in resets:
                assert np.array_equal(obs[i], seqs[i][k][2]), (i, k)
        if steps:
            # the kernel steps every lane: lanes without a step op at k are restored afterwards
            acts = torch.zeros(n, 15, dtype=torch.float32)
            for i in steps:
                acts[i] = torch.from_numpy(seqs[i][k][1])
            # snapshot non-stepping lanes' state so the extra step does not perturb them
            snap = env.state.clone()
            obs, rew, te, tr = env.step(acts.to(dev))
            obs, rew, te, tr = obs.cpu().numpy(), rew.cpu().numpy(), te.cpu().numpy(), tr.cpu().numpy()
            keep = torch.zeros(n, dtype=torch.bool)
            keep[steps] = True
            _restore_lanes(env, snap, ~keep)
            for i in steps:
                eo, er, et, etr = seqs[i][k][2]
                assert np.array_equal(obs[i], eo), (i, k)
                assert math.isclose(rew[i], er, rel_tol=REW_RTOL, abs_tol=1e-15)
                assert (bool(te[i]), bool(tr[i])) == (bool(et), bool(etr))


def _restore_lanes(env, snap, lanes_mask):
    """Copy the SoA columns of `lanes_mask` lanes back from a snapshot slab."""
    lay, n = env.layout, env.num_envs
    m = lanes_mask.to(env.device)
    for off, rows, dt in ((lay.jp, 15, torch.float32), (lay.jv, 15, torch.float32), (lay.op, 3, torch.float64),
                          (lay.ov, 3, torch.float32), (lay.flags, 1, torch.int32), (lay.step_count, 1, torch.int32)):
        nbytes = rows * n * torch.empty((), dtype=dt).element_size()
        cur = env.state[off:off + nbytes].view(dt).view(rows, n)
        old = snap[off:off + nbytes].view(dt).view(rows, n)
        cur[:, m] = old[:, m]


def test_large_batch_vs_oracle(pkg):
    """N=4099 lanes (ragged), device-RNG resets, random actions incl. out-of-range values;
    32 sampled lanes re-simulated by the CPU oracle from the device's own reset state."""
    n, T = 4099, 60
    C = pkg.experiments.CurriculumConfig
    env = pkg.envs.VecEnv(n, reward_type="dense", seed=1234)
    cfgs = [C.variable(), C.easy(), C.hard(), C.medium()]
    idx = (np.arange(n) % 4).astype(np.int32)
    env.set_curricula(cfgs, env_index=idx)
    obs0 = env.reset().cpu().numpy()
    rng = np.random.default_rng(5)
    lanes = np.sort(rng.choice(n, 32, replace=False))
    lanes[-1] = n - 1  # the tail lane
    # oracle envs initialised from the device reset state
    jp = env.joint_positions.cpu().numpy()
    op = env.object_position.cpu().numpy()
    size = env.object_size.cpu().numpy()
    fric = env.friction_coefficient.cpu().numpy()
    mass = env.object_mass.cpu().numpy()
    orcs = {}
    for i in lanes:
        cur = OracleCurriculum(object_size=size[i], friction_coefficient=fric[i], object_mass=mass[i])
        o = OracleEnv(cur=cur, dense=True)
        d = np.full(21, np.nan)
        d[:15] = jp[:, i].astype(np.float64)
        d[18:21] = op[:, i]
        o.reset(d)
        assert np.array_equal(o.obs(), obs0[i])
        orcs[i] = o
    acts = rng.uniform(-1.4, 1.4, size=(T, n, 15)).astype(np.float32)
    acts[:, :, ::4] = np.where(rng.random((T, n, 4)) < 0.5, -1.0, 1.0)[..., :acts[:, :, ::4].shape[-1]]
    dev = env.device
    for t in range(T):
        ob, rw, te, tr = env.step(torch.from_numpy(acts[t]).to(dev))
        ob, rw, te, tr = ob.cpu().numpy(), rw.cpu().numpy(), te.cpu().numpy(), tr.cpu().numpy()
        for i in lanes:
            eo, er, et, etr = orcs[i].step(acts[t, i])
            assert np.array_equal(ob[i], eo), (t, i)
            assert math.isclose(rw[i], er, rel_tol=REW_RTOL, abs_tol=1e-15)
            assert (bool(te[i]), bool(tr[i])) == (et, etr)
    # size-independent properties over all lanes
    assert np.all(np.abs(ob[:, :15]) <= 1.0)
    assert np.all(ob[:, 33] == 1.0) and np.all(ob[:, 34:37] == 0.0)
    ncon = ob[:, 40:45].sum(1)
    assert np.array_equal(te.astype(bool), ncon >= 3)
    assert np.all(env.step_count.cpu().numpy() == T)


def test_streaming_step_policy_is_bit_identical(pkg, monkeypatch):
    """Large batches stream with non-temporal stores (N >= 2^20) and loads (N >= 2^21;
    dxrl_env.hip kNtStoreMinEnvs / kNtLoadMinEnvs); every policy variant (0 plain, 1 nt stores,
    2 nt loads, 3 both) gives the default-policy kernel's results bit for bit, and sampled lanes
    match the oracle."""
    n, T = (1 << 21) + 37, 4
    dev = torch.device("cuda:0")
    envs = []
    for v in ("0", "1", "2", "3"):
        e = pkg.envs.VecEnv(n, curriculum_config=pkg.experiments.CurriculumConfig.variable(), reward_type="dense",
                            seed=77, device=dev)
        e.reset(write_obs=False)
        envs.append((v, e))
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    outs = {}
    for t in range(T):
        a = (torch.rand(n, 15, generator=g, device=dev) * 2.6 - 1.3).contiguous()
        for v, e in envs:
            monkeypatch.setenv("DXRL_STEP_VARIANT", v)
            outs[v] = [x.clone() for x in e.step(a)]
        for v in ("1", "2", "3"):
            for x, y in zip(outs["0"], outs[v]):
                assert torch.equal(x, y), v
    monkeypatch.delenv("DXRL_STEP_VARIANT")
    e = envs[3][1]
    a = (torch.rand(n, 15, generator=g, device=dev) * 2.6 - 1.3).contiguous()
    jp, jv = e.joint_positions.cpu().numpy(), e.joint_velocities.cpu().numpy()
    op, ov = e.object_position.cpu().numpy(), e.object_velocity.cpu().numpy()
    size, fric, mass = (x.cpu().numpy() for x in (e.object_size, e.friction_coefficient, e.object_mass))
    flags, tcount = e.flags.cpu().numpy(), e.step_count.cpu().numpy()
    ob, rw, te, tr = (x.cpu().numpy() for x in e.step(a))  # default policy at this N: both non-temporal
    an = a.cpu().numpy()
    for i in [0, 1, 255, 256, 4097, n // 2, n - 1]:
        o = OracleEnv(cur=OracleCurriculum(object_size=size[i], friction_coefficient=fric[i], object_mass=mass[i]))
        o.jp, o.jv = [np.float32(x) for x in jp[:, i]], [np.float32(x) for x in jv[:, i]]
        o.op, o.ov = [float(x) for x in op[:, i]], [np.float32(x) for x in ov[:, i]]
        o.op_is_f32 = bool(flags[i] & (1 << 17))
        o.contacts = [int((flags[i] >> f) & 1) for f in range(5)]
        o.prev = [int((flags[i] >> (8 + f)) & 1) for f in range(5)] if flags[i] & (1 << 16) else None
        o.t = int(tcount[i])
        o.size, o.fric, o.mass = float(size[i]), float(fric[i]), float(mass[i])
        eo, er, et, etr = o.step(an[i])
        assert np.array_equal(ob[i], eo) and math.isclose(rw[i], er, rel_tol=REW_RTOL, abs_tol=1e-15)
        assert (bool(te[i]), bool(tr[i])) == (et, etr)


def test_device_rng_reset_ranges_and_sticky(pkg):
    n = 2048
    C = pkg.experiments.CurriculumConfig
    env = pkg.envs.VecEnv(n, reward_type="dense", seed=7)
    env.set_curriculum(C.variable())
    env.reset()
    jp = env.joint_positions.cpu().numpy()
    assert jp.min() >= -0.1 and jp.max() <= 0.1 and jp.std() > 0.05
    s = env.object_size.cpu().numpy()
    assert s.min() >= 0.03 and s.max() <= 0.07 and len(np.unique(s)) > n // 2
    op0 = env.object_position.cpu().numpy()
    assert op0[2].min() >= 0.05 and op0[2].max() <= 0.2
    assert np.array_equal(op0, op0.astype(np.float32).astype(np.float64))  # f32-rounded at reset
    acts = torch.zeros(n, 15, dtype=torch.float32, device=env.device)
    for _ in range(5):
        env.step(acts)
    op1 = env.object_position.cpu().numpy()
    env.reset()
    op2 = env.object_position.cpu().numpy()
    assert np.array_equal(op2, op1.astype(np.float32).astype(np.float64))  # sticky (quirk 1)
    assert not np.array_equal(env.joint_positions.cpu().numpy(), jp)  # fresh counter-based draws


LEARNER_CASES = G.meta()["learner_cases"]


@pytest.mark.parametrize("case", LEARNER_CASES, ids=lambda c: f"l{c['index']}-{c['cfg']}")
def test_facade_run_episode_simple_learner(pkg, case):
    """Reference loop (run_episode) on the facade with the device SimpleLearner."""
    z = G.learner_case(case["index"])
    env = pkg.envs.DexterousManipulationEnv(reward_type=case["reward"],
                                            curriculum_config=_curriculum(pkg, case["curriculum"]),
                                            max_episode_steps=case.get("max_episode_steps", 200))
    env.np_random = _pcg(case["env_seed"])
    np.random.seed(case["learner_seed"])
    pol = pkg.policies.SimpleLearner(env.action_space, learning_rate=case["lr"])
    for e in range(case["episodes"]):
        s, n, tot = pkg.training.run_episode(env, pol, max_steps=case["max_steps"])
        assert (s, n) == (False, z["ep_steps"][e])
        assert math.isclose(tot, z["ep_return"][e], rel_tol=REW_RTOL)
    assert np.array_equal(pol.mean_action, z["final_mean"])


def _learner_groups():
    groups = {}
    for c in LEARNER_CASES:
        key = (c["reward"], c.get("max_episode_steps", 200), c["max_steps"], c["lr"])
        groups.setdefault(key, []).append(c)
    return sorted(groups.items(), key=lambda kv: str(kv[0]))


@pytest.mark.parametrize("key,group", _learner_groups(), ids=lambda x: str(x) if isinstance(x, tuple) else "")
def test_fused_rollout_matches_reference(pkg, key, group):
    """dxrl_rollout_simple in parity mode: each reference learner case is one
    lane; the rollout runs in uneven chunks and must reproduce every
    run_episode of the reference (lengths, returns, success=False)."""
    reward, mes, ms, lr = key
    n = len(group)
    env = pkg.envs.VecEnv(n, reward_type=reward, max_episode_steps=mes)
    env.set_curricula([_curriculum(pkg, c["curriculum"]) for c in group], env_index=np.arange(n, dtype=np.int32))
    learner = pkg.policies.VecSimpleLearner(n, learning_rate=lr, device=env.device)
    streams = pkg.training.ReferenceStreams(env, [c["env_seed"] for c in group], [c["learner_seed"] for c in group])
    ro = pkg.training.SimpleLearnerRollout(env, learner, max_steps=ms, streams=streams)
    idx = np.arange(n)
    ro.start(env_index=idx)
    zs = [G.learner_case(c["index"]) for c in group]
    total = max(int(z["ep_steps"].sum()) for z in zs)
    got = {i: [] for i in range(n)}
    done = 0
    for chunk in (37, 1, 64, 200, 500, 500):
        if done >= total:
            break
        rec = ro.run(chunk, env_index=idx)
        assert rec.dropped == 0
        assert np.all(np.diff(rec.end_step) >= 0)
        for k in range(len(rec)):
            got[int(rec.env_id[k])].append((int(rec.steps[k]), float(rec.total_reward[k]), bool(rec.success[k])))
        done += chunk
    for i, (c, z) in enumerate(zip(group, zs)):
        eps = got[i][:c["episodes"]]
        assert len(eps) == c["episodes"], (c["index"], len(got[i]))
        for e, (steps, ret, succ) in enumerate(eps):
            assert steps == z["ep_steps"][e] and not succ
            assert math.isclose(ret, z["ep_return"][e], rel_tol=REW_RTOL), (c["index"], e)


def test_random_policy_plumbing_c1(pkg):
    """Config C1: RandomPolicy + run_episode on the facade (default curriculum)."""
    z = G.npz("learner_traces")
    rp = G.meta()["random_policy"]
    env = pkg.envs.DexterousManipulationEnv(reward_type="dense", max_episode_steps=rp["max_episode_steps"])
    env.np_random = _pcg(rp["env_seed"])
    pol = pkg.policies.RandomPolicy(env.action_space, seed=42)
    env.action_space.seed(rp["box_seed"])
    for e in range(rp["episodes"]):
        s, n, tot = pkg.training.run_episode(env, pol)
        assert (s, n) == (bool(z["rp_ep_success"][e]), z["rp_ep_steps"][e])
        assert math.isclose(tot, z["rp_ep_return"][e], rel_tol=REW_RTOL)


def test_device_rollout_throughput_mode_invariants(pkg):
    """Philox mode at the bench size: episode bookkeeping invariants."""
    n, T = 4096, 200
    C = pkg.experiments.CurriculumConfig
    env = pkg.envs.VecEnv(n, reward_type="dense", seed=3)
    env.set_curriculum(C.easy())
    learner = pkg.policies.VecSimpleLearner(n, seed=11, device=env.device)
    ro = pkg.training.SimpleLearnerRollout(env, learner, record_cap=T)
    ro.start()
    rec = ro.run(T)
    assert rec.dropped == 0 and len(rec) > 0
    assert np.all(rec.steps >= 1) and np.all(rec.steps <= 200)
    assert not rec.success.any()  # training success rule (quirk 3)
    # per env: lengths of finished episodes + the open episode == T
    counts = ro.ep_count.cpu().numpy()
    open_len = env.step_count.cpu().numpy()
    sums = np.zeros(n, np.int64)
    np.add.at(sums, rec.env_id, rec.steps)
    assert np.array_equal(sums + open_len, np.full(n, T))
    assert counts.sum() == len(rec)
    m = learner.mean_action.cpu().numpy()
    assert np.abs(m).max() <= 0.5 and np.abs(m).max() > 0


NOISE_CASES = G.meta()["noise_cases"]


@pytest.mark.parametrize("ci", range(len(NOISE_CASES)))
def test_noise_wrapper_on_facade(pkg, ci):
    """CombinedNoiseWrapper over the facade, driven as RobustnessTester does."""
    c = NOISE_CASES[ci]
    z = G.noise_case(ci)
    cfg = _curriculum(pkg, G.meta()["host"]["configs"][c["cfg"]])
    base = pkg.envs.DexterousManipulationEnv(curriculum_config=cfg, reward_type="dense", max_episode_steps=200)
    env = pkg.evaluation.CombinedNoiseWrapper(base, c["obs_std"], c["dyn_std"], seed=c["seed"])
    for e in range(c["episodes"]):
        obs, _ = env.reset(seed=c["seed"] + e)
        assert np.array_equal(obs, z["reset_obs"][e])
        for t in range(z["length"][e]):
            obs, r, te, tr, _ = env.step(z["actions"][e, t])
            assert np.array_equal(obs, z["obs"][e, t]), (e, t)
            assert math.isclose(r, z["reward"][e, t], rel_tol=REW_RTOL, abs_tol=1e-15)


def test_heldout_table_on_device(pkg):
    """Config C4: HeldOutObjectSet (heldout_objects.py:39-189) as the device curricula table --
    env i resets to held-out object i % 20 exactly (scalar size/mass/friction, f64 in the slab)."""
    ev = pkg.evaluation
    hs = ev.HeldOutObjectSet(pkg.experiments.CurriculumConfig.hard(), seed=42)
    n = 1000
    env = pkg.envs.VecEnv(n, reward_type="dense", seed=9)
    cfgs, idx = hs.native_table(n)
    env.set_curricula(cfgs, env_index=idx)
    env.reset(write_obs=False)
    size, mass, fric = (t.cpu().numpy() for t in (env.object_size, env.object_mass, env.friction_coefficient))
    for i in (0, 1, 19, 20, 537, n - 1):
        o = hs.heldout_objects[i % len(hs.heldout_objects)]
        assert (size[i], mass[i], fric[i]) == (o.size, o.mass, o.friction), i
    # a step on the held-out table advances without error and keeps the per-env objects
    env.step(torch.zeros(n, 15, device=env.device))
    assert np.array_equal(env.object_size.cpu().numpy(), size)


def test_c4_full_size_heldout_vs_oracle(pkg):
    """Config C4 at its full size: 8192 envs on the HeldOutObjectSet(hard, seed=42) table
    (heldout_objects.py:46-143), device-RNG resets, 40 steps of random actions.  28 sampled
    lanes (incl. the first, the tail and every 256-env workgroup boundary tested) re-simulated by
    the CPU oracle from the device's own reset state; a second env with the same seed must
    reproduce the whole batch bit-for-bit (the streams depend only on seed and env id)."""
    n, T = 8192, 40
    hs = pkg.evaluation.HeldOutObjectSet(pkg.experiments.CurriculumConfig.hard(), seed=42)
    cfgs, idx = hs.native_table(n)
    envs = []
    for _ in range(2):
        e = pkg.envs.VecEnv(n, reward_type="dense", seed=77)
        e.set_curricula(cfgs, env_index=idx)
        e.reset()
        envs.append(e)
    env, twin = envs
    assert torch.equal(env.obs, twin.obs)
    obs0 = env.obs.cpu().numpy()
    jp, op = env.joint_positions.cpu().numpy(), env.object_position.cpu().numpy()
    size, fric, mass = (t.cpu().numpy() for t in (env.object_size, env.friction_coefficient, env.object_mass))
    rng = np.random.default_rng(8192)
    lanes = np.unique(np.concatenate([[0, 255, 256, 4095, 4096, n - 1], rng.choice(n, 22, replace=False)]))
    orcs = {}
    for i in lanes:
        o = hs.heldout_objects[i % len(hs.heldout_objects)]
        assert (size[i], mass[i], fric[i]) == (o.size, o.mass, o.friction), i
        orc = OracleEnv(cur=OracleCurriculum(object_size=size[i], friction_coefficient=fric[i],
                                             object_mass=mass[i]), dense=True)
        d = np.full(21, np.nan)
        d[:15] = jp[:, i].astype(np.float64)
        d[18:21] = op[:, i]
        orc.reset(d)
        assert np.array_equal(orc.obs(), obs0[i])
        orcs[i] = orc
    dev = env.device
    for t in range(T):
        a = torch.from_numpy(rng.uniform(-1.2, 1.2, size=(n, 15)).astype(np.float32)).to(dev)
        ob, rw, te, tr = (x.cpu().numpy() for x in env.step(a))
        tw = twin.step(a)
        assert torch.equal(twin.obs, env.obs) and torch.equal(twin.reward, env.reward), t
        an = a.cpu().numpy()
        for i in lanes:
            eo, er, et, etr = orcs[i].step(an[i])
            assert np.array_equal(ob[i], eo), (t, i)
            assert math.isclose(rw[i], er, rel_tol=REW_RTOL, abs_tol=1e-15), (t, i)
            assert (bool(te[i]), bool(tr[i])) == (et, etr), (t, i)
        assert np.array_equal(tw[2].cpu().numpy(), te)
    assert np.all(np.abs(ob[:, :15]) <= 1.0)
    assert np.array_equal(te.astype(bool), ob[:, 40:45].sum(1) >= 3)
    assert np.all(env.step_count.cpu().numpy() == T)
