"""CPU: host-side surfaces against the reference's golden data (configs,
curriculum scheduler traces, held-out object tables) and host plumbing."""
import json
import math

import numpy as np
import pytest

import golden_io as G
import dexterous_rl_manipulation_amd as dx
from dexterous_rl_manipulation_amd import evaluation as ev
from dexterous_rl_manipulation_amd import experiments as ex

HOST = G.meta()["host"]


def _rec(cfg):
    out = {}
    for k, v in cfg.to_dict().items():
        out[k] = [float(x) for x in v] if isinstance(v, (tuple, list)) else (None if v is None else float(v))
    out["_float64_scalars"] = [k for k in ("object_size", "object_mass", "friction_coefficient")
                               if isinstance(getattr(cfg, k), np.floating)]
    return out


@pytest.mark.parametrize("name", ["easy", "medium", "hard", "variable", "default"])
def test_curriculum_presets_match_reference(name):
    assert _rec(ex.CurriculumConfig.named(name)) == HOST["configs"][name]
    if name != "default":  # config_{easy,medium,hard,variable}.json load to the same curriculum
        js = HOST["configs"][f"json:config_{name}.json"]
        assert _rec(ex.CurriculumConfig.from_dict(js)) == HOST["configs"][name]


def test_curriculum_json_round_trip(tmp_path):
    c = ex.CurriculumConfig.variable()
    p = tmp_path / "c.json"
    c.to_json(str(p))
    c2 = ex.CurriculumConfig.from_json(str(p))
    assert _rec(c2) == _rec(c)
    with pytest.raises(TypeError):
        ex.CurriculumConfig.from_dict({"bogus": 1})


def test_curriculum_samplers_draw_order():
    rng = np.random.default_rng(5)
    c = ex.CurriculumConfig.variable()
    got = [c.get_object_size(rng), c.get_object_mass(rng), c.get_friction_coefficient(rng)]
    rng2 = np.random.default_rng(5)
    exp = [float(rng2.uniform(0.03, 0.07)), float(rng2.uniform(0.05, 0.15)), float(rng2.uniform(0.3, 0.7))]
    assert got == exp
    assert ex.CurriculumConfig.easy().get_object_size(rng) == 0.08  # no range: no draw, constant


@pytest.mark.parametrize("name", ["default", "quick_test"])
def test_named_experiment_configs_match_reference_json(name):
    ref = HOST["configs"][f"json:config_{name}.json"]
    got = ex.load_named_config(name).to_dict()
    assert json.loads(json.dumps(got)) == ref


def test_experiment_config_strict_and_round_trip(tmp_path):
    c = ex.ExperimentConfig.quick_test()
    p = tmp_path / "e.json"
    c.to_json(str(p))
    c2 = ex.load_config(str(p))
    assert c2.to_dict() == c.to_dict()
    d = c.to_dict()
    d["training"]["unknown"] = 1
    with pytest.raises(TypeError):
        ex.ExperimentConfig.from_dict(d)
    with pytest.raises(FileNotFoundError):
        ex.load_config("/nonexistent/x.json")
    with pytest.raises(ValueError):
        ex.SeedVarianceConfig(seeds=[1, 2]).validate()


@pytest.mark.parametrize("ci", range(3))
def test_curriculum_scheduler_trace(ci):
    sc = HOST["scheduler"][ci]
    s = ex.CurriculumScheduler(ex.CurriculumConfig.easy(), ex.CurriculumConfig.hard(),
                               success_rate_threshold=sc["thr"], window_size=sc["window"],
                               min_episodes_before_progression=sc["min_eps"], progression_steps=sc["steps"])
    for k, (a, b) in enumerate(zip(sc["successes"], sc["steps_seq"])):
        assert s.update(a, b) == sc["progressed"][k], k
        assert s.get_difficulty_level() == sc["levels"][k]
        assert _rec(s.get_current_config()) == sc["configs"][k], k
    st = json.loads(json.dumps(s.get_statistics()))
    assert st == sc["statistics"]


def test_step_based_scheduler_trace():
    sc = HOST["step_scheduler"]
    s = ex.StepBasedScheduler(ex.CurriculumConfig.easy(), ex.CurriculumConfig.hard(),
                              step_milestones=sc["milestones"])
    prog = [bool(s.update(False, b)) for b in sc["steps_seq"]]
    assert prog == sc["progressed"]
    assert json.loads(json.dumps(s.get_statistics())) == sc["statistics"]
    assert _rec(s.get_current_config()) == sc["final"]


def test_interpolated_friction_is_numpy_float64_on_device_row():
    s = ex.CurriculumScheduler(ex.CurriculumConfig.easy(), ex.CurriculumConfig.hard())
    c = s._interpolate_config(0.4)
    assert isinstance(c.friction_coefficient, np.floating)
    assert _rec(c) == HOST["configs"]["interp"]
    # the NEP-50 f64 damping flag travels to the kernel row only for numpy scalars without a range
    pytest.importorskip("torch")
    assert c.to_native().friction_is_f64_scalar == 1
    assert ex.CurriculumConfig.easy().to_native().friction_is_f64_scalar == 0


@pytest.mark.parametrize("hi", range(4))
def test_heldout_object_tables(hi):
    h = HOST["heldout"][hi]
    s = ev.HeldOutObjectSet(ex.CurriculumConfig.named(h["cfg"]), num_heldout_objects=h["n"], seed=h["seed"])
    assert [list(s.eval_size_range), list(s.eval_mass_range), list(s.eval_friction_range)] == \
        [h["eval_size_range"], h["eval_mass_range"], h["eval_friction_range"]]
    assert [[o.size, o.mass, o.friction] for o in s.heldout_objects] == h["objects"]
    for i, rec in enumerate(h["eval_configs"]):
        assert _rec(s.get_eval_config(i)) == rec  # index bit-exact incl. wrap-around (i % n)
    st = json.loads(json.dumps(s.get_statistics()))
    assert st == json.loads(json.dumps(h["statistics"]))
    cfgs, idx = s.native_table(25)
    assert list(idx) == [i % h["n"] for i in range(25)] and len(cfgs) == h["n"]


def test_training_objects_and_separation():
    objs = ev.generate_training_objects(ex.CurriculumConfig.variable(), num_samples=50, seed=42)
    assert [[o.size, o.mass, o.friction] for o in objs] == HOST["training_objects"]
    h = ev.HeldOutObjectSet(ex.CurriculumConfig.variable(), num_heldout_objects=20, seed=123)
    assert h.verify_separation(objs)
    assert not h.verify_separation(h.heldout_objects[:1])


def test_episode_records_order_and_host_streams():
    from dexterous_rl_manipulation_amd.training import EpisodeRecords
    r = EpisodeRecords(env_id=np.array([0, 1]), end_step=np.array([3, 3]), total_reward=np.array([1.0, 2.0]),
                       steps=np.array([4, 4]), success=np.array([False, False]))
    assert len(r) == 2 and r.dropped == 0


def test_package_surface_imports_without_gpu():
    assert dx.CurriculumConfig is ex.CurriculumConfig
    from dexterous_rl_manipulation_amd import envs
    with pytest.raises(Exception):
        envs.VecEnv(4)  # no GPU here: the product refuses to run (no CPU fallback)


def test_scheduler_update_batch_equals_sequential_updates():
    """CurriculumScheduler.update_batch (the trainer's per-iteration feed) == one update() per
    episode (curriculum_scheduler.py:116-153): same lists, totals, progression points, history."""
    from dexterous_rl_manipulation_amd.experiments import CurriculumConfig as CC, CurriculumScheduler
    rng = np.random.default_rng(0)
    for _ in range(200):
        kw = dict(success_rate_threshold=float(rng.choice([0.0, 0.3, 0.5, 0.7])),
                  min_episodes_before_progression=int(rng.integers(0, 40)), window_size=int(rng.integers(1, 25)),
                  progression_steps=int(rng.integers(1, 7)))
        a, b = CurriculumScheduler(CC.easy(), CC.hard(), **kw), CurriculumScheduler(CC.easy(), CC.hard(), **kw)
        p = rng.random()
        for _ in range(int(rng.integers(1, 6))):
            m = int(rng.integers(0, 60))
            s, st = rng.random(m) < p, rng.integers(1, 200, m)
            assert any([a.update(bool(x), int(y)) for x, y in zip(s, st)]) == b.update_batch(s, st)
            assert a.episode_successes == b.episode_successes and a.episode_steps == b.episode_steps
            assert (a.total_steps, a.total_episodes) == (b.total_steps, b.total_episodes)
            assert type(b.total_episodes) is int and type(b.total_steps) is int
            assert a.current_difficulty_level == b.current_difficulty_level
            assert a.progression_history == b.progression_history and a.current_config == b.current_config


def _sched_kw(rng):
    return dict(success_rate_threshold=float(rng.choice([0.0, 0.3, 0.5, 0.7])),
                min_episodes_before_progression=int(rng.integers(0, 40)), window_size=int(rng.integers(1, 25)),
                progression_steps=int(rng.integers(1, 7)))


def test_step_based_update_batch_equals_sequential_updates():
    """StepBasedScheduler.update_batch == one update() per episode: a milestone fires at the
    first episode whose running step total reaches it, at most one per episode
    (curriculum_scheduler.py:276-335)."""
    from dexterous_rl_manipulation_amd.experiments import CurriculumConfig as CC, StepBasedScheduler
    rng = np.random.default_rng(1)
    for _ in range(200):
        ms = sorted(rng.integers(0, 3000, int(rng.integers(1, 6))).tolist())
        a = StepBasedScheduler(CC.easy(), CC.hard(), ms, **_sched_kw(rng))
        b = StepBasedScheduler(CC.easy(), CC.hard(), ms, **_sched_kw(rng))
        b.__dict__.update({k: v for k, v in a.__dict__.items() if not isinstance(v, list)})
        for _ in range(int(rng.integers(1, 6))):
            m = int(rng.integers(0, 40))
            s, st = rng.random(m) < 0.5, rng.integers(1, 200, m)
            assert any([a.update(bool(x), int(y)) for x, y in zip(s, st)]) == b.update_batch(s, st)
            assert a.episode_successes == b.episode_successes and a.episode_steps == b.episode_steps
            assert (a.total_steps, a.total_episodes, a.current_milestone_idx) == \
                (b.total_steps, b.total_episodes, b.current_milestone_idx)
            assert a.progression_history == b.progression_history and a.current_config == b.current_config


def test_window_history_matches_full_history():
    """history="window" keeps the last window_size episodes and counters only: totals,
    statistics and progression history equal the full-history scheduler's."""
    from dexterous_rl_manipulation_amd.experiments import CurriculumConfig as CC, CurriculumScheduler
    rng = np.random.default_rng(2)
    for _ in range(100):
        kw = _sched_kw(rng)
        a = CurriculumScheduler(CC.easy(), CC.hard(), **kw)
        b = CurriculumScheduler(CC.easy(), CC.hard(), history="window", **kw)
        for _ in range(int(rng.integers(1, 6))):
            m = int(rng.integers(0, 60))
            s, st = rng.random(m) < rng.random(), rng.integers(1, 200, m)
            if rng.random() < 0.5:
                assert a.update_batch(s, st) == b.update_batch(s, st)
            else:
                assert any([a.update(bool(x), int(y)) for x, y in zip(s, st)]) == \
                    any([b.update(bool(x), int(y)) for x, y in zip(s, st)])
            assert a.get_statistics() == b.get_statistics()
            assert b.episode_successes == a.episode_successes[-kw["window_size"]:]
            assert len(b.episode_steps) <= kw["window_size"]


@pytest.mark.parametrize("history", ["window", "full"])
def test_device_summary_replay_equals_sequential_updates(history):
    """The dxrl_sched_scan contract (restated in tests/sched_reference.py) replayed by
    CurriculumScheduler.apply_device_summary == one update() per episode in (end step,
    global env id) order, over random multi-rank code tapes and several batches."""
    import sched_reference as SR
    from dexterous_rl_manipulation_amd.experiments import CurriculumConfig as CC, CurriculumScheduler
    rng = np.random.default_rng(3)
    for _ in range(150):
        kw = _sched_kw(rng)
        a = CurriculumScheduler(CC.easy(), CC.hard(), **kw)
        b = CurriculumScheduler(CC.easy(), CC.hard(), history=history, **kw)
        w = kw["window_size"]
        for _ in range(int(rng.integers(1, 5))):
            world, T, n = int(rng.integers(1, 4)), int(rng.integers(1, 9)), int(rng.integers(1, 12))
            p_end, p_succ = rng.random(), rng.random()
            lens = rng.integers(1, 300, (world, T, n))
            codes = np.where(rng.random((world, T, n)) < p_end, (lens << 1) | (rng.random((world, T, n)) < p_succ), 0)
            ep = SR.order_codes(codes)
            want = any([a.update(bool(c & 1), int(c >> 1)) for c in ep])
            P = b.remaining_progressions(64)
            tail_in = [int(x) for x in b.episode_successes[-w:]]
            r = SR.scan(codes, w, kw["success_rate_threshold"], kw["min_episodes_before_progression"],
                        b.total_episodes, P, tail_in)
            got = b.apply_device_summary(r["episodes"], r["steps"], r["successes"], r["candidates"],
                                         r["tail"][len(r["tail"]) - min(w, len(ep)):],
                                         episode_codes=ep if history == "full" else None)
            assert want == got
            assert a.get_statistics() == b.get_statistics()
            assert b.episode_successes == a.episode_successes[-len(b.episode_successes):]
            assert b.episode_steps == a.episode_steps[-len(b.episode_steps):]
            if history == "full":
                assert a.episode_successes == b.episode_successes and a.episode_steps == b.episode_steps


def test_minibatch_bounds_cut_on_whole_rounds():
    """PPO minibatch slices (trainer.minibatch_bounds): whole 128 x CU rounds split as evenly
    as possible, covering [0, M) exactly, each a multiple of 32 samples."""
    from dexterous_rl_manipulation_amd.trainer import minibatch_bounds
    rnd = 128 * 256
    assert minibatch_bounds(819200, 4, rnd) == [0, 7 * rnd, 13 * rnd, 19 * rnd, 25 * rnd]
    assert minibatch_bounds(819200, 1, rnd) == [0, 819200]
    assert minibatch_bounds(819200, 5, rnd) == [0, 5 * rnd, 10 * rnd, 15 * rnd, 20 * rnd, 25 * rnd]
    for M, B in ((8192, 4), (100000 - 100000 % 32, 3), (1638400, 16), (96 * 32, 2)):
        b = minibatch_bounds(M, B, rnd)
        assert b[0] == 0 and b[-1] == M and len(b) == B + 1
        assert all(y > x and (y - x) % 32 == 0 for x, y in zip(b, b[1:])), b


def test_reward_plugin_overrides_are_rejected():
    """A plugin whose compute() (or a dense _compute_* term) is overridden cannot run inside the
    fused step kernels: resolve_plugin raises TypeError instead of silently computing the
    built-in reward (envs/manipulation_env.py:64-73 accepts any object with compute()).
    Weight-only subclasses and the built-ins resolve."""
    from dexterous_rl_manipulation_amd import rewards as R

    class Custom(R.RewardShaping):
        def compute(self, *a, **k):
            return {"total": 42.0}

    class CustomTerm(R.RewardShaping):
        def _compute_distance_reward(self, tips, op):
            return 0.0

    class CustomSparse(R.SparseReward):
        def compute(self, *a, **k):
            return {"total": 1.0}

    class Heavier(R.RewardShaping):
        def __init__(self):
            super().__init__(distance_weight=2.0)

    class DuckTyped:
        native_kind = "dense"
        weights = (1.0, 0.5, 0.3, 0.2)

        def compute(self, *a, **k):
            return {"total": 0.0}

    for bad in (Custom(), CustomTerm(), CustomSparse(), DuckTyped(), object()):
        with pytest.raises(TypeError):
            R.resolve_plugin("dense", bad)
    assert R.resolve_plugin("dense", Heavier())[:2] == ("dense", (2.0, 0.5, 0.3, 0.2))
    assert R.resolve_plugin("dense", None)[0] == "dense"
    assert R.resolve_plugin("sparse", None)[0] == "sparse"
    assert R.resolve_plugin("sparse", R.SparseReward())[0] == "sparse"


def test_reward_plugin_compute_has_no_cpu_fallback():
    """compute() runs on the GPU only (dxrl_reward_compute): without a GPU it raises."""
    import torch

    from dexterous_rl_manipulation_amd import _native as N
    from dexterous_rl_manipulation_amd import rewards as R
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(N.NativeError):
        R.RewardShaping().compute(np.zeros(15, np.float32), np.zeros((5, 3)), np.zeros(3), np.zeros(5, np.float32), 5, 3)
    with pytest.raises(N.NativeError):
        R.SparseReward().compute(None, None, None, np.zeros(5, np.float32), 5, 3)


def test_sqrt_below_margin_test_is_exact():
    """csrc/dxrl_device.h sqrt_below: the contact test sqrt_rn(x) < t decided on x against
    q (1 -+ 2^-40) with q = fl(t t), the exact root only inside that window.  Restated in f64
    NumPy (IEEE, correctly rounded sqrt) on values straddling the threshold: the margin
    branches never disagree with the root.  Also min_f sqrt_rn(x_f) == sqrt_rn(min_f x_f)."""
    rng = np.random.default_rng(3)
    t = rng.uniform(0.003, 0.5, 200_000) * 1.5
    q = t * t
    rel = rng.choice([1e-18, 1e-16, 1e-14, 1e-12, 1e-9, 1e-6, 1e-3, 0.3], t.size) * rng.choice([-1, 1], t.size)
    x = np.concatenate([q * (1 + rel), q, np.nextafter(q, 0), np.nextafter(q, 1), (np.nextafter(t, 0)) ** 2,
                        (np.nextafter(t, 1)) ** 2])
    tt = np.concatenate([t] * 6)
    qq = tt * tt
    truth = np.sqrt(x) < tt
    lo, hi = x < qq * (1.0 - 2.0 ** -40), x > qq * (1.0 + 2.0 ** -40)
    assert not (lo & hi).any()
    assert truth[lo].all() and not truth[hi].any()
    fast = np.where(lo, True, np.where(hi, False, truth))
    assert np.array_equal(fast, truth)
    xs = rng.uniform(0, 0.1, (100_000, 5))
    assert np.array_equal(np.sqrt(xs).min(1), np.sqrt(xs.min(1)))


def test_div_by_five_without_division_is_correctly_rounded():
    """csrc/dxrl_device.h div_f: f32(f64(x) * 0.2) == x / 5 in IEEE f32 (correctly rounded, as
    NumPy's f32 division and -fhip-fp32-correctly-rounded-divide-sqrt give) -- every f32 of the
    binades [2^-8, 2^5) (the closure / stability arguments lie in [0, 15]) plus a log-uniform
    sample over the normal range."""
    f32 = np.float32
    m = np.arange(1 << 23, dtype=np.uint32)
    for e in range(-8, 5):
        x = ((m | np.uint32(127 + e) << np.uint32(23)).view(np.float32))
        assert np.array_equal((x.astype(np.float64) * 0.2).astype(f32), x / f32(5)), e
    rng = np.random.default_rng(1)
    x = (2.0 ** rng.uniform(-126, 127, 4_000_000)).astype(f32)
    assert np.array_equal((x.astype(np.float64) * 0.2).astype(f32), x / f32(5))
