"""GPU: the policy-gradient learner against the plain-PyTorch fp32 reference
(tests/pg_reference.py, bf16 rounding emulated at the pipeline's storage
points) and against the CPU env oracle.  Parity vs the reference repository
is unpinned: it has no network learner."""
import math

import numpy as np
import pytest
import torch

import pg_reference as R
from oracle.dx_oracle import OracleCurriculum, OracleEnv

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pkg():
    import dexterous_rl_manipulation_amd as d
    from dexterous_rl_manipulation_amd import envs, trainer  # noqa: F401
    return d


def make(pkg, n=128, T=16, **kw):
    env = pkg.envs.VecEnv(n, curriculum_config=pkg.CurriculumConfig.variable(), reward_type="dense", seed=3)
    cfg = pkg.trainer.TrainerConfig(horizon=T, seed=1, ent_coef=0.01, **kw)
    tr = pkg.trainer.PGTrainer(env, cfg)
    env.reset(write_obs=False)
    return env, tr


def test_param_count_and_pack(pkg):
    env, tr = make(pkg)
    T = pkg.trainer
    assert T.LOGICAL_PARAMS == 159_263
    torch.cuda.synchronize()
    P, B = tr.params, tr.packed
    for name in ("W1a", "W2a", "W3a", "W1c", "W2c", "W3c"):
        blk = tr.block(name)
        got = B[T.BF[name]:T.BF[name] + blk.numel()].view_as(blk)
        assert torch.equal(got, blk.to(torch.bfloat16))
    for net in "ac":
        W2, W3 = tr.block(f"W2{net}"), tr.block(f"W3{net}")
        W2T = B[T.BF[f"W2{net}T"]:T.BF[f"W2{net}T"] + T.W2T].view(256, 256)
        W3T = B[T.BF[f"W3{net}T"]:T.BF[f"W3{net}T"] + T.W3T].view(256, 32)
        assert torch.equal(W2T, W2[:, :256].T.to(torch.bfloat16))
        assert torch.equal(W3T, W3[:, :256].T.to(torch.bfloat16))
    # padding stays zero; logstd initialised
    assert tr.block("W1a")[:, 46:].abs().sum() == 0 and tr.block("W3a")[15:].abs().sum() == 0
    assert torch.all(P[T.OFF["logstd"]:T.OFF["logstd"] + 15] == -0.5)


def test_rollout_tape_matches_env_oracle(pkg):
    n, T = 96, 24
    env, tr = make(pkg, n, T)
    jp, op = env.joint_positions.cpu().numpy(), env.object_position.cpu().numpy()
    size, mass, fric = (t.cpu().numpy() for t in (env.object_size, env.object_mass, env.friction_coefficient))
    tr.rollout()
    torch.cuda.synchronize()
    obs = tr.obs_rm.float().cpu().numpy()
    act = tr.act.cpu().numpy()
    rew, done = tr.rew.cpu().numpy(), tr.done.cpu().numpy()
    assert np.all(obs[:, 45] == 1.0) and np.all(obs[:, 46:] == 0.0)
    checked = 0
    for i in range(n):
        o = OracleEnv(cur=OracleCurriculum(object_size=size[i], object_mass=mass[i], friction_coefficient=fric[i]))
        d = np.full(21, np.nan)
        d[:15], d[18:21] = jp[:, i], op[:, i]
        ob = o.reset(d)
        assert np.array_equal(obs[i, :45], torch.from_numpy(ob).to(torch.bfloat16).float().numpy())
        for t in range(T):
            m = t * n + i
            ob, r, te, tr_ = o.step(act[m, :15])
            assert rew[m] == np.float32(r), (i, t)
            d_ = te or tr_ or o.t >= env.max_episode_steps
            assert bool(done[m]) == d_, (i, t)
            checked += 1
            if d_:
                break
            assert np.array_equal(obs[(t + 1) * n + i, :45], torch.from_numpy(ob).to(torch.bfloat16).float().numpy())
    assert checked >= n * 2


def _learner_pass(tr):
    """One iteration without the optimizer step, on either learner path."""
    for name in tr.phases():
        if name != "optimizer_step":
            getattr(tr, name)()
    torch.cuda.synchronize()


@pytest.mark.parametrize("fused", [True, False])
def test_rollout_policy_matches_training_forward(pkg, fused):
    """The in-kernel actor (rollout) and the training actor (fused kernel or GEMM chain)
    agree bit for bit: ratios are exactly 1 on the first update (kl 0, nothing clipped)."""
    env, tr = make(pkg, 256, 32, fused=fused)
    _learner_pass(tr)
    s = tr.loss_stats()
    assert s["clip_frac"] == 0.0 and abs(s["approx_kl"]) < 1e-9


@pytest.mark.parametrize("n,T,fused", [(256, 32, True), (256, 32, False), (773, 32, True), (5, 32, True),
                                       (100, 40, False)])
def test_iteration_matches_torch_reference(pkg, n, T, fused):
    """One learner pass vs the torch fp32 restatement; 773 x 32: ragged last 128-sample tile and
    24 dW2 slabs of 32-33 chunks; 5 x 32: one partial tile, one slab."""
    env, tr = make(pkg, n, T, fused=fused)
    _learner_pass(tr)
    cfg = dict(gamma=tr.cfg.gamma, lam=tr.cfg.lam, clip_eps=tr.cfg.clip_eps, vf_coef=tr.cfg.vf_coef,
               ent_coef=tr.cfg.ent_coef)
    g_ref, info = R.loss_and_grads(tr.params.clone(), tr.obs_rm, tr.act, tr.logp, tr.rew, tr.done, n, T, cfg,
                                   bf16=True)
    M = n * T
    # Hidden activations are stored in bf16; the torch reference accumulates in a different
    # order, so ~5% of values sit on the other side of a bf16 rounding tie (one bf16 ulp,
    # 2^-8 relative, of one of 256 hidden units) -> abs tolerances of a few 1e-3 on V/mu.
    torch.testing.assert_close(tr.V[0], info["V"], rtol=1e-2, atol=3e-3)
    if not fused:  # the fused kernel never materialises mu
        torch.testing.assert_close(tr.mu[:, :15], info["mu"][:, :15], rtol=1e-2, atol=1e-3)
    torch.testing.assert_close(tr.adv, info["adv"], rtol=1e-2, atol=5e-3)
    torch.testing.assert_close(tr.ret, info["ret"], rtol=1e-2, atol=5e-3)
    assert (tr.V[0] - info["V"]).norm() / info["V"].norm() < 2e-3
    assert math.isclose(tr.stats[2].item(), info["mean"].item(), rel_tol=1e-2, abs_tol=1e-4)
    assert math.isclose(tr.stats[4].item(), info["std"].item(), rel_tol=1e-3)
    T_ = pkg.trainer
    for name in ("W1a", "W2a", "W3a", "W1c", "W2c", "W3c"):
        got, ref = tr.block(name, tr.grads), R.unpack(g_ref)[name]
        rel = (got - ref).norm() / ref.norm().clamp_min(1e-12)
        cos = torch.nn.functional.cosine_similarity(got.flatten(), ref.flatten(), dim=0)
        assert rel < 2e-2 and cos > 0.9998, (name, rel.item(), cos.item())
    ls = slice(T_.OFF["logstd"], T_.OFF["logstd"] + 15)
    torch.testing.assert_close(tr.grads[ls], g_ref[ls], rtol=1e-3, atol=1e-6)
    assert M == tr.M
    # fp64 truth: no block, nor V / adv, further from it than 1.5 x the bf16 torch reference
    R.fp64_pin(tr.grads, tr.V[0], tr.adv, tr.params.clone(), tr.obs_rm, tr.act, tr.logp, tr.rew, tr.done, n, T, cfg,
               g_ref, info)


@pytest.mark.parametrize("n,T,h1_recompute", [(256, 32, True), (96, 33, True), (256, 32, False), (96, 33, False)])
def test_fused_learner_matches_gemm_chain(pkg, n, T, h1_recompute):
    """dxrl_pg_fused (one pass per network) == the layer-by-layer GEMM chain: same bf16
    storage points, so only f32 accumulation order differs (96 * 33 = 3168: ragged last
    128-sample tile).  h1_recompute: dW2 with H1 recomputed from obs on chip vs read back
    from the HBM copy."""
    if (n * T) % 32:
        pytest.skip("trainer needs num_envs * horizon % 32 == 0")
    _, tf = make(pkg, n, T, fused=True, h1_recompute=h1_recompute)
    _, tu = make(pkg, n, T, fused=False)
    tf.rollout()
    tu.rollout()
    torch.cuda.synchronize()
    assert torch.equal(tf.obs_rm, tu.obs_rm) and torch.equal(tf.act, tu.act)
    for name in [x for x in tf.phases() if x not in ("rollout", "optimizer_step")]:
        getattr(tf, name)()
    for name in [x for x in tu.phases() if x not in ("rollout", "optimizer_step")]:
        getattr(tu, name)()
    torch.cuda.synchronize()
    torch.testing.assert_close(tf.V[0], tu.V[0], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(tf.adv, tu.adv, rtol=1e-4, atol=1e-5)
    assert math.isclose(tf.stats[4].item(), tu.stats[4].item(), rel_tol=1e-5)
    for name in ("W1a", "W2a", "W3a", "W1c", "W2c", "W3c"):
        a, b = tf.block(name, tf.grads), tu.block(name, tu.grads)
        rel = (a - b).norm() / b.norm().clamp_min(1e-12)
        assert rel < 1e-3, (name, rel.item())
    T_ = pkg.trainer
    ls = slice(T_.OFF["logstd"], T_.OFF["logstd"] + 32)
    torch.testing.assert_close(tf.grads[ls], tu.grads[ls], rtol=1e-4, atol=1e-7)
    lf, lu = tf.loss_stats(), tu.loss_stats()
    for k in ("policy_loss", "value_mse", "clip_frac", "approx_kl"):
        assert math.isclose(lf[k], lu[k], rel_tol=1e-4, abs_tol=1e-7), (k, lf[k], lu[k])


@pytest.mark.parametrize("n,T", [(256, 32), (773, 32), (5, 32), (1, 96)])
def test_h1_recompute_is_bit_exact(pkg, n, T):
    """dW2 from H1 recomputed on chip (k_wgrad_l1) == dW2 from the H1 HBM copy, bit for bit:
    the recompute repeats the learner forward's L1 exactly and both contractions sum in the
    same order.  Sizes: 32 chunks per workgroup; 32-33 (ragged over 24 splits); 5 and 3 chunks
    in one workgroup (shorter than the chunk ring's look-ahead)."""
    grads = []
    for rec in (True, False):
        _, tr = make(pkg, n, T, fused=True, h1_recompute=rec, pair_learner=False)
        tr.rollout()
        for name in [x for x in tr.phases() if x not in ("rollout", "optimizer_step")]:
            getattr(tr, name)()
        torch.cuda.synchronize()
        grads.append(tr.grads.clone())
    assert torch.equal(grads[0], grads[1])


@pytest.mark.parametrize("n,T,mb", [(256, 32, 1), (2048, 32, 4), (773, 64, 1)])
def test_paired_learner_equals_two_passes(pkg, n, T, mb):
    """dxrl_pg_fused_pair (both train passes, ONE dW2 launch for both networks, ONE reduction
    launch) == two dxrl_pg_fused calls with the same dW2 split count, bit for bit: every
    gradient block, the loss sums, and (PPO minibatch slices) every minibatch's gradients."""
    outs = []
    for paired in (True, False):
        _, tr = make(pkg, n, T, minibatches=mb)
        assert tr.paired
        if not paired:
            tr.paired = False
            tr.splits = tr.pair_splits  # the paired step's per-network split count
            tr.kpartial = torch.zeros(tr.splits + 16, 256, 288, device=tr.dev)
        tr.rollout()
        tr.critic_values()
        tr.advantages()
        b = tr.minibatch_bounds()
        got = []
        for k in range(mb):
            tr._mb = (b[k], b[k + 1] - b[k])
            tr.train_passes()
            torch.cuda.synchronize()
            got.append((tr.grads.clone(), tr.fused_loss.clone()))
        outs.append(got)
    for (ga, la), (gb, lb) in zip(*outs):
        assert torch.equal(ga, gb)
        assert torch.equal(la, lb)


@pytest.mark.parametrize("n,T,mb,paired,diag", [(4096, 32, 1, True, 0), (773, 32, 1, True, 0),
                                               (2048, 32, 4, True, 0), (1001, 32, 1, False, 0),
                                               (8192, 8, 1, True, 0), (5, 32, 1, True, 0),
                                               (1000, 32, 1, True, 1024)])
def test_stored_h2_equals_recomputed(pkg, n, T, mb, paired, diag):
    """TrainerConfig.reuse_h2: the actor's layer-2 activations written by the rollout (16- and
    32-env kernels) and the critic's written by the critic-values pass, read by the first train
    passes under those weights (LDS-DMA into the H2 tile), give the recomputing passes' results bit
    for bit: V, every minibatch's gradients, loss sums and dH2 of both networks.  Ragged tiles, PPO
    slices, the per-network path, 8192 envs (the 32-env rollout kernel's tape), the 32-env kernel
    forced on a ragged 1000 envs (diag 1024: a partial last workgroup), and fewer rows than one
    tile."""
    outs = []
    for reuse in (True, False):
        _, tr = make(pkg, n, T, minibatches=mb, reuse_h2=reuse)
        tr.diag_flags = diag
        if not paired:
            tr.paired = False
        tr.rollout()
        tr.critic_values()
        tr.advantages()
        torch.cuda.synchronize()
        if reuse:  # what the passes below read
            assert tr._h2c_fresh == (mb == 1)
            assert tr._h2a_fresh  # both the 16- and the 32-env rollout kernels write the tape
        b = tr.minibatch_bounds()
        got = [tr.V.clone()]
        for k in range(mb):
            tr._mb = (b[k], b[k + 1] - b[k])
            tr.train_passes()
            torch.cuda.synchronize()
            rows = b[k + 1] - b[k]
            got.append((tr.grads.clone(), tr.fused_loss.clone(), tr.dH2[:rows].clone(),
                        tr.dH2c[:rows].clone() if tr.dH2c is not None and paired else None))
        outs.append(got)
    va, vb = outs[0][0], outs[1][0]
    assert torch.equal(va, vb)
    for x, y in zip(outs[0][1:], outs[1][1:]):
        for u, w in zip(x, y):
            if u is not None:
                assert torch.equal(u, w)


def test_stored_h2_is_refreshed_after_every_update(pkg):
    """PPO 2 x 2 through iteration(): only the first train pair of an iteration reads the stored
    activations (the optimiser step makes them stale); parameters after two iterations equal the
    recomputing trainer's bit for bit."""
    params = []
    for reuse in (True, False):
        _, tr = make(pkg, 1024, 32, epochs=2, minibatches=2, reuse_h2=reuse)
        for _ in range(2):
            tr.iteration()
            assert not tr._h2a_fresh and not tr._h2c_fresh
        torch.cuda.synchronize()
        params.append(tr.params.clone())
    assert torch.equal(params[0], params[1])


@pytest.mark.parametrize("n,T,mb,max_norm", [(256, 32, 1, 0.5), (2048, 32, 4, 1e-3), (512, 32, 1, 1e6)])
def test_reduction_gnorm_partials_match_sumsq_path(pkg, n, T, mb, max_norm):
    """One rank, paired step (TrainerConfig.fused_gnorm): the grad-norm partials written by the
    pair's reduction (dxrl_pg_fused_pair_gnorm) sum to k_sumsq's squared norm of the finished
    gradient to f64 rounding; the gradients are dxrl_pg_fused_pair's bit for bit; and
    dxrl_pg_adam_step on those partials == dxrl_pg_optimizer_step on the same state -- bit for
    bit when the clip is not engaged (max_norm 1e6), to f32 rounding of the clip scale when it
    is.  PPO minibatch slices included."""
    from dexterous_rl_manipulation_amd import _native as N
    _, tr = make(pkg, n, T, minibatches=mb, max_grad_norm=max_norm)
    assert tr.paired and tr.gn_partial is not None
    T_, c, s = pkg.trainer, tr.cfg, N.stream_of(tr.dev)
    tr.rollout()
    tr.critic_values()
    tr.advantages()
    b = tr.minibatch_bounds()
    engaged = []
    for k in range(mb):
        tr._mb = (b[k], b[k + 1] - b[k])
        gp = tr.gn_partial
        tr.gn_partial = None
        tr.train_passes()  # dxrl_pg_fused_pair
        g_plain = tr.grads.clone()
        tr.gn_partial = gp
        tr.train_passes()  # dxrl_pg_fused_pair_gnorm
        torch.cuda.synchronize()
        assert torch.equal(tr.grads, g_plain) and tr._gn_blocks == gp.numel(), k
        part, g2 = torch.zeros_like(tr.partial), torch.zeros_like(tr.gnorm2)
        N.call("dxrl_pg_grad_sumsq", tr.dev.index, N.ptr(tr.grads), T_.NPARAMS, N.ptr(part), N.ptr(g2), s)
        outs = []
        for fold in (True, False):
            po, m1o, m2o = (torch.empty_like(t) for t in (tr.params, tr.m1, tr.m2))
            packed, n2 = tr.packed.clone(), torch.zeros_like(tr.gnorm2)
            args = (N.ptr(tr.params), N.ptr(tr.grads), N.ptr(tr.m1), N.ptr(tr.m2), N.ptr(po), N.ptr(m1o), N.ptr(m2o),
                    T_.NPARAMS, c.lr, c.betas[0], c.betas[1], c.adam_eps, tr.step_count + 1, c.max_grad_norm)
            if fold:
                N.call("dxrl_pg_adam_step", tr.dev.index, *args, N.ptr(tr.gn_partial), tr._gn_blocks, N.ptr(n2),
                       N.ptr(packed), s)
            else:
                N.call("dxrl_pg_optimizer_step", tr.dev.index, *args, N.ptr(torch.zeros_like(tr.partial)), N.ptr(n2),
                       N.ptr(packed), s)
            torch.cuda.synchronize()
            outs.append((po, m1o, m2o, packed, n2.item()))
        (pa, ma, va, ka, na), (pb, mbb, vb, kb, nb) = outs
        assert math.isclose(na, g2.item(), rel_tol=1e-12) and math.isclose(nb, g2.item(), rel_tol=1e-12), k
        assert math.isclose(float(tr.gn_partial.sum()), na, rel_tol=1e-12), k
        engaged.append(math.sqrt(na) > max_norm)
        if not engaged[-1]:
            assert torch.equal(pa, pb) and torch.equal(ma, mbb) and torch.equal(va, vb), k
            assert torch.equal(ka.view(torch.int16), kb.view(torch.int16)), k
        else:
            torch.testing.assert_close(ma, mbb, rtol=1e-6, atol=1e-12)
            torch.testing.assert_close(va, vb, rtol=1e-6, atol=1e-18)
            torch.testing.assert_close(pa, pb, rtol=1e-6, atol=1e-9)
            torch.testing.assert_close(ka.float(), kb.float(), rtol=1e-2, atol=1e-6)
        tr.optimizer_step()  # the trainer's own step: the fold, the same partials
        torch.cuda.synchronize()
        assert tr._gn_blocks == 0 and tr.gnorm2.item() == na, k
        assert torch.equal(tr.params, pa) and torch.equal(tr.packed.view(torch.int16), ka.view(torch.int16)), k
    if max_norm == 1e-3:
        assert all(engaged), engaged
    if max_norm == 1e6:
        assert not any(engaged), engaged


@pytest.mark.parametrize("n,T", [(773, 32), (4096, 200), (96, 1)])
def test_values_kernel_equals_layer_by_layer_pass(pkg, n, T, monkeypatch):
    """The critic-values kernel pipelined across tiles (k_pg_values: next X stored under L2, next L1
    beside the value head) == the layer-by-layer forward instantiation bit for bit, at a ragged
    row count (773 x 33 rows), the full bench shape and a single tile per workgroup."""
    _, tr = make(pkg, n, T)
    tr.rollout()
    tr.critic_values()
    torch.cuda.synchronize()
    v_pipe = tr.V.clone()
    tr.V.fill_(float("nan"))
    monkeypatch.setenv("DXRL_FWD_LAYERED", "1")
    tr.critic_values()
    torch.cuda.synchronize()
    assert torch.equal(tr.V, v_pipe)
    assert torch.isfinite(v_pipe[0, :(T + 1) * n]).all()


def test_adam_matches_manual(pkg):
    env, tr = make(pkg, 64, 16)
    tr.grads.normal_(0, 1e-3)
    p0 = tr.params.clone()
    g = tr.grads.clone()
    tr.optimizer_step()
    torch.cuda.synchronize()
    c = tr.cfg
    norm = g.double().norm().item()
    scale = c.max_grad_norm / (norm + 1e-6) if norm > c.max_grad_norm else 1.0
    gs = g * scale
    m1 = (1 - c.betas[0]) * gs
    m2 = (1 - c.betas[1]) * gs * gs
    upd = c.lr * (m1 / (1 - c.betas[0])) / (torch.sqrt(m2 / (1 - c.betas[1])) + c.adam_eps)
    torch.testing.assert_close(tr.params, p0 - upd, rtol=1e-5, atol=1e-7)


def test_training_runs_and_moves(pkg):
    env, tr = make(pkg, 512, 64)
    p0 = tr.params.clone()
    for _ in range(5):
        tr.iteration()
    torch.cuda.synchronize()
    assert torch.isfinite(tr.params).all() and not torch.equal(tr.params, p0)
    s = tr.loss_stats()
    assert all(math.isfinite(v) for v in s.values())
    st = tr.episode_stats()
    assert st["env_steps"] == 512 * 64


def test_episode_records_match_tape(pkg):
    """Per-episode records (feeds CurriculumScheduler, curriculum_scheduler.py:116) agree with the
    done/reward tape: one record per done flag, end step, length, f64 return."""
    n, T = 64, 40
    cap = T  # at most one episode ends per step
    env, tr = make(pkg, n, T, max_steps=9, record_cap=cap)
    tr.rollout()
    torch.cuda.synchronize()
    rew, done = tr.rew.cpu().numpy().reshape(T, n), tr.done.cpu().numpy().reshape(T, n).astype(bool)
    rec = tr.episode_records()
    assert rec.dropped == 0 and len(rec) == int(done.sum())
    assert np.all(np.diff(rec.end_step) >= 0)
    for i in range(n):
        ends = np.nonzero(done[:, i])[0]
        sel = rec.env_id == i
        assert np.array_equal(rec.end_step[sel], ends)
        starts = np.concatenate([[0], ends[:-1] + 1])
        assert np.array_equal(rec.steps[sel], ends - starts + 1)
        want = np.array([rew[s:e + 1, i].astype(np.float64).sum() for s, e in zip(starts, ends)])
        np.testing.assert_allclose(rec.total_reward[sel], want, rtol=1e-5, atol=1e-6)
    assert int(rec.success.sum()) == int(tr.ep_succ.sum().item())


def test_curriculum_scheduler_hook(pkg):
    """A progression decided on this iteration's records lands in the device curricula table."""
    n, T = 64, 40
    env, tr = make(pkg, n, T, max_steps=9, record_cap=T, success_rule="training")
    C = pkg.CurriculumConfig
    sched = pkg.experiments.CurriculumScheduler(C.easy(), C.hard(), success_rate_threshold=0.0,
                                                min_episodes_before_progression=1, window_size=1,
                                                progression_steps=4)
    tr.attach_curriculum(sched)
    tr.iteration()
    torch.cuda.synchronize()
    assert sched.total_episodes == int(tr.ep_count.sum().item()) > 0
    assert sched.get_difficulty_level() == 1.0
    cur = env.curriculum_configs[0]
    assert float(cur.object_size) == float(sched.get_current_config().object_size)


@pytest.mark.parametrize("std", [0.0, 0.05])
def test_fused_observation_noise(pkg, std):
    """Config C5: NoisyObservationWrapper (robustness_tests.py:140-171) fused into the rollout:
    the policy sees obs + N(0, std^2) per element; the env state is untouched."""
    n = 256
    env, tr = make(pkg, n, 1, obs_noise_std=std)
    clean = env.observe().clone()
    jp0 = env.joint_positions.clone()
    tr.rollout()
    torch.cuda.synchronize()
    seen = tr.obs_rm[:n, :45].float()
    res = (seen - clean).cpu().numpy().ravel()
    if std == 0.0:
        np.testing.assert_array_equal(seen.cpu().numpy(), clean.to(torch.bfloat16).float().cpu().numpy())
    else:
        assert abs(res.mean()) < 3e-3 and 0.047 < res.std() < 0.053
        # independent per element and per env
        assert abs(np.corrcoef(res.reshape(n, 45)[:, 0], res.reshape(n, 45)[:, 1])[0, 1]) < 0.2
    assert not torch.equal(env.joint_positions, jp0)  # the env stepped on its own state


@pytest.mark.parametrize("std", [0.0, 0.05])
def test_fused_dynamics_noise(pkg, std):
    """Config C5: NoisyDynamicsWrapper (robustness_tests.py:174-211): the env integrates
    clip(a + N(0, std^2), -1, 1) while the tape keeps the policy's action a.  The applied
    action is recovered from the joint-velocity update jv' = 0.9 jv + 0.1 a (ME:203)."""
    n = 256
    env, tr = make(pkg, n, 1, dyn_noise_std=std)
    jv0 = env.joint_velocities.clone().double()
    tr.rollout()
    torch.cuda.synchronize()
    jv1 = env.joint_velocities.double()
    applied = ((jv1 - np.float32(0.9) * jv0) / np.float32(0.1)).T.cpu().numpy()  # [n, 15]
    policy = np.clip(tr.act[:n, :15].cpu().numpy(), -1, 1)
    live = tr.done[:n].cpu().numpy() == 0  # an env that finished at this step was auto-reset
    assert live.sum() > n // 2
    applied, policy = applied[live], policy[live]
    res = applied - policy
    if std == 0.0:
        assert np.abs(res).max() < 1e-4
    else:
        inner = res[(np.abs(applied) < 0.999) & (np.abs(policy) < 0.8)]
        assert inner.size > 500
        assert abs(inner.mean()) < 4e-3 and 0.046 < inner.std() < 0.054


@pytest.mark.parametrize("cur,n,noise", [("easy", 96, 0.0), ("variable", 100, 0.0), ("hard", 64, 0.05),
                                         ("variable", 4100, 0.05)])
def test_lane_split_rollout_matches_64_env_kernel(pkg, cur, n, noise):
    """k_pg_rollout_ws (default: 16 envs x 16 lanes, env waves + aux twin waves, 8 waves),
    k_pg_rollout (diag 16: one lane per env) and k_pg_rollout_e8 (diag 1024: 32 envs x 8 lanes,
    the kernel of >= 32 envs per CU) share every Philox stream and every op: tapes, episode
    records and env state are equal bit for bit (auto-resets, observation / dynamics noise, a
    ragged last workgroup)."""
    T = 24
    outs = []
    for diag in (16, 0, 1024):
        env = pkg.envs.VecEnv(n, curriculum_config=pkg.CurriculumConfig.named(cur), reward_type="dense", seed=11)
        cfg = pkg.trainer.TrainerConfig(horizon=T, seed=5, max_steps=13, record_cap=T, obs_noise_std=noise,
                                        dyn_noise_std=noise)
        tr = pkg.trainer.PGTrainer(env, cfg)
        env.reset(write_obs=False)
        tr.diag_flags = diag
        for _ in range(2):
            tr.rollout()
            tr.iteration_index += 1
        torch.cuda.synchronize()
        outs.append([t.clone() for t in (tr.obs_rm, tr.act, tr.logp, tr.rew, tr.done, tr.ep_ret, tr.ep_count,
                                          tr.rec_return, tr.rec_length, tr.rec_end, env.joint_positions,
                                          env.joint_velocities, env.object_position, env.object_velocity, env.flags,
                                          env.step_count, env.object_size, env.friction_coefficient)])
    for other in outs[1:]:
        for k, (a, b) in enumerate(zip(outs[0], other)):
            assert torch.equal(a, b), k


def test_minibatch_gradients_sum_to_full_batch(pkg):
    """Time-contiguous minibatches (pointer offsets into the tape, same kernels): each pass is
    the gradient of the mean loss over its own samples (scale 1 / its rows), so the mean of the
    two halves' gradients equals the full batch's -- log_std included (its entropy bonus
    enters every pass once) -- and loss_stats() of each pass is per sample of that pass."""
    env, tr = make(pkg, 256, 32, minibatches=2)
    for name in ("rollout", "critic_values", "advantages"):
        getattr(tr, name)()
    M = tr.M
    got, losses = [], []
    for mb in ((0, M // 2), (M // 2, M // 2), (0, M)):
        tr._mb = mb
        tr.actor_train()
        tr.critic_train()
        torch.cuda.synchronize()
        got.append(tr.grads.clone())
        losses.append(tr.loss_stats())
    T_ = pkg.trainer
    ls = slice(T_.OFF["logstd"], T_.OFF["logstd"] + 15)
    for name in ("W1a", "W2a", "W3a", "W1c", "W2c", "W3c"):
        a = 0.5 * (tr.block(name, got[0]) + tr.block(name, got[1]))
        b = tr.block(name, got[2])
        assert ((a - b).norm() / b.norm()).item() < 1e-5, name
    torch.testing.assert_close(0.5 * (got[0][ls] + got[1][ls]), got[2][ls], rtol=1e-5, atol=1e-7)
    for k in ("policy_loss", "value_mse"):
        assert abs(0.5 * (losses[0][k] + losses[1][k]) - losses[2][k]) <= 1e-5 * max(1.0, abs(losses[2][k])), k


def test_unequal_minibatch_gradients_weight_to_full_batch(pkg):
    """Unequal time-contiguous slices M/4, M/2, M/4 at a ragged size (772 x 32: the slices start
    inside a 128-sample tile, end on a partial one, and deal 32-33 dW2 chunks per slab):
    sum_k rows_k / M x grad_k == the full-batch gradient.  Power-of-two row ratios keep the
    per-sample loss scale's bf16 roundings identical across passes, so the tolerance is f32
    summation order only (with a 1/9600-vs-1/24736 split the scaled bf16 head gradients round
    differently and W1a moves by ~4e-3)."""
    env, tr = make(pkg, 772, 32)
    for name in ("rollout", "critic_values", "advantages"):
        getattr(tr, name)()
    M = tr.M
    q = M // 4
    assert q % 32 == 0 and q % 128
    slices = ((0, q), (q, 2 * q), (3 * q, q), (0, M))
    got = []
    for mb in slices:
        tr._mb = mb
        tr.actor_train()
        tr.critic_train()
        torch.cuda.synchronize()
        got.append(tr.grads.clone())
    w = [rows / M for _, rows in slices[:3]]
    for name in ("W1a", "W2a", "W3a", "W1c", "W2c", "W3c"):  # biases ride in each block's extra column
        a = sum(wk * tr.block(name, g) for wk, g in zip(w, got))
        b = tr.block(name, got[3])
        assert ((a - b).norm() / b.norm()).item() < 1e-5, name
    ls = slice(pkg.trainer.OFF["logstd"], pkg.trainer.OFF["logstd"] + 15)
    torch.testing.assert_close(sum(wk * g[ls] for wk, g in zip(w, got)), got[3][ls], rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("n", [256, 772])
def test_ppo_epochs_engage_the_clip(pkg, n):
    """epochs x minibatches > 1: after the first Adam step the ratio leaves 1, so the later
    minibatches see a nonzero KL and (with a large learning rate) clipped samples.  772 x 32:
    minibatch slices that start inside a 128-sample tile."""
    env, tr = make(pkg, n, 32, epochs=3, minibatches=4, lr=3e-3)
    assert "ppo_updates" in tr.phases()
    p0 = tr.params.clone()
    tr.iteration()
    torch.cuda.synchronize()
    s = tr.loss_stats()
    assert tr.step_count == 12 and not torch.equal(tr.params, p0)
    assert abs(s["approx_kl"]) > 1e-7 and s["clip_frac"] > 0.0, s
    assert all(math.isfinite(v) for v in s.values())


def test_fused_optimizer_step_equals_three_launch_path(pkg):
    """dxrl_pg_optimizer_step (grad-norm partials + one clipped-Adam-and-pack launch, output to
    the spare buffers) == dxrl_pg_grad_sumsq + dxrl_pg_adam + dxrl_pg_pack_weights bit for bit:
    master, both moments, the grad norm and every bf16 packed copy, over three steps with the
    clip engaged and not."""
    from dexterous_rl_manipulation_amd import _native as N
    env, tr = make(pkg, 64, 16)
    T_ = pkg.trainer
    c = tr.cfg
    p, m1, m2 = tr.params.clone(), tr.m1.clone(), tr.m2.clone()
    packed, part, g2 = tr.packed.clone(), torch.zeros_like(tr.partial), torch.zeros_like(tr.gnorm2)
    gen = torch.Generator(device=tr.dev).manual_seed(5)
    s = N.stream_of(tr.dev)
    for k, sd in enumerate((1e-3, 10.0, 1e-2)):  # 10.0: global norm far above max_grad_norm
        g = torch.randn(T_.NPARAMS, generator=gen, device=tr.dev) * sd
        tr.grads.copy_(g)
        tr.optimizer_step()
        N.call("dxrl_pg_grad_sumsq", tr.dev.index, N.ptr(g), T_.NPARAMS, N.ptr(part), N.ptr(g2), s)
        N.call("dxrl_pg_adam", tr.dev.index, N.ptr(p), N.ptr(g), N.ptr(m1), N.ptr(m2), T_.NPARAMS, c.lr,
               c.betas[0], c.betas[1], c.adam_eps, k + 1, N.ptr(g2), c.max_grad_norm, s)
        N.call("dxrl_pg_pack_weights", tr.dev.index, N.ptr(p), N.ptr(packed), s)
        torch.cuda.synchronize()
        assert torch.equal(tr.params, p) and torch.equal(tr.m1, m1) and torch.equal(tr.m2, m2), k
        assert torch.equal(tr.gnorm2, g2), k
        assert torch.equal(tr.packed.view(torch.int16), packed.view(torch.int16)), k


def test_optimizer_step_matches_torch_clip_and_adam(pkg):
    """dxrl_pg_optimizer_step against PyTorch's own optimiser, not another kernel path:
    torch.nn.utils.clip_grad_norm_(max_norm) + torch.optim.Adam(lr, betas, eps) in fp32 over
    three steps (clipping engaged on the second).  The kernel writes the bias-corrected
    denominator as sqrt(v / bc2) + eps where torch writes sqrt(v) / sqrt(bc2) + eps, so the
    masters agree to fp32 rounding, not bit for bit; the squared global norm is an f64 sum in
    both."""
    env, tr = make(pkg, 64, 16)
    T_ = pkg.trainer
    c = tr.cfg
    ref = torch.nn.Parameter(tr.params.clone())
    opt = torch.optim.Adam([ref], lr=c.lr, betas=tuple(c.betas), eps=c.adam_eps)
    gen = torch.Generator(device=tr.dev).manual_seed(11)
    for k, sd in enumerate((1e-3, 10.0, 1e-2)):
        g = torch.randn(T_.NPARAMS, generator=gen, device=tr.dev) * sd
        tr.grads.copy_(g)
        tr.optimizer_step()
        ref.grad = g.clone()
        norm = torch.nn.utils.clip_grad_norm_([ref], c.max_grad_norm)
        opt.step()
        torch.cuda.synchronize()
        assert math.isclose(math.sqrt(tr.gnorm2.item()), float(g.double().norm()), rel_tol=1e-9), k
        assert math.isclose(math.sqrt(tr.gnorm2.item()), float(norm), rel_tol=1e-6), k
        st = opt.state[ref]
        torch.testing.assert_close(tr.m1, st["exp_avg"], rtol=1e-5, atol=1e-9)
        torch.testing.assert_close(tr.m2, st["exp_avg_sq"], rtol=1e-5, atol=1e-12)
        torch.testing.assert_close(tr.params, ref.detach(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("n,T,p_done", [(100, 1, 0.1), (64, 7, 0.0), (4096, 25, 0.05), (96, 33, 0.3),
                                        (4096, 200, 0.02), (130, 256, 0.0), (70, 300, 0.05),
                                        # many envs, short horizons: the partial buffer's worst cases
                                        (8192, 32, 0.05), (6000, 8, 0.1), (65536, 1, 0.2),
                                        # past the LDS staging limit: the k_gae fallback
                                        (200, 800, 0.01)])
def test_gae_lds_scan_matches_sequential_reference(pkg, n, T, p_done):
    """dxrl_pg_gae (k_gae_lds: the horizon staged in LDS by the whole workgroup, the recurrence a
    16-lane segmented wavefront scan per env; k_gae, one sequential chain per env, past T = 600)
    gives pg_reference.gae's adv / ret (the restatement of the kernel's op order, scan included)
    bit for bit, and the moments (count, mean, M2) a two-pass f64 reduction's to 1e-9.
    Ragged env counts, no dones and dense dones, horizons from 1 to 800.  `partial` is sized by
    dxrl_pg_gae_partial_doubles exactly, with a NaN canary block behind it that must survive
    (one Moments triple per workgroup; the header once documented half of that)."""
    from dexterous_rl_manipulation_amd import _native as N
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(n * 1000 + T)
    rew = torch.randn(T * n, generator=g, device=dev)
    V = torch.randn((T + 1) * n, generator=g, device=dev) * 3.0
    done = (torch.rand(T * n, generator=g, device=dev) < p_done).to(torch.uint8)
    adv, ret = torch.empty_like(rew), torch.empty_like(rew)
    need = N.gae_partial_doubles(n, T)
    assert need == 3 * ((n + 15) // 16)
    canary = 4096
    part = torch.full((need + canary,), float("nan"), dtype=torch.float64, device=dev)
    stats = torch.zeros(8, dtype=torch.float64, device=dev)
    N.call("dxrl_pg_gae", 0, N.ptr(rew), N.ptr(done), N.ptr(V), n, T, 0.99, 0.95, N.ptr(adv), N.ptr(ret),
           N.ptr(part), N.ptr(stats), N.stream_of(dev))
    torch.cuda.synchronize()
    assert torch.isnan(part[need:]).all(), "dxrl_pg_gae wrote past dxrl_pg_gae_partial_doubles"
    a_ref, r_ref = R.gae(rew, done, V, n, T, 0.99, 0.95)
    assert torch.equal(adv, a_ref) and torch.equal(ret, r_ref)
    a = adv.double()
    assert stats[0].item() == n * T
    assert math.isclose(stats[2].item(), a.mean().item(), rel_tol=1e-9, abs_tol=1e-12)
    if n * T > 1:
        assert math.isclose(stats[4].item(), a.std().item(), rel_tol=1e-9)
