"""Generate the golden parity fixtures from the reference implementation.

Run ONLY in the build container (the reference never travels to the GPU box):

    cd /tmp && python3 -B /root/repo/tests/golden/gen_golden.py

It imports the reference read-only from /root/reference (nothing is written
there: bytecode writing is disabled and no file under /root/reference is
opened for writing).  gymnasium is not installed in this image, so an
in-memory stand-in for the two gymnasium pieces the reference uses
(``gymnasium.Env`` seeding and ``spaces.Box``) is registered in
``sys.modules``; it follows gymnasium>=0.29 ``utils.seeding.np_random``
(``Generator(PCG64(SeedSequence(seed)))``) and the bounded branch of
``Box.sample``.  This stand-in is test infrastructure, not reference source.

Outputs (committed): tests/golden/*.npz and tests/golden/*.json — inputs and
expected outputs only.
"""
import json
import os
import sys
import types

import numpy as np

sys.dont_write_bytecode = True
REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------
# gymnasium stand-in (seeding + Box), registered before the reference imports
# --------------------------------------------------------------------------
def _pcg(seed):
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))


def install_gym_standin():
    gym = types.ModuleType("gymnasium")
    spaces = types.ModuleType("gymnasium.spaces")

    class Env:
        metadata = {}
        _np_random = None

        @property
        def np_random(self):
            if self._np_random is None:
                self._np_random = _pcg(None)
            return self._np_random

        @np_random.setter
        def np_random(self, value):
            self._np_random = value

        def reset(self, *, seed=None, options=None):
            if seed is not None:
                self._np_random = _pcg(seed)

        def close(self):
            pass

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.dtype = np.dtype(dtype)
            self.shape = tuple(shape)
            self.low = np.full(self.shape, low, dtype=self.dtype)
            self.high = np.full(self.shape, high, dtype=self.dtype)
            self._np_random = None

        @property
        def np_random(self):
            if self._np_random is None:
                self._np_random = _pcg(None)
            return self._np_random

        def seed(self, seed=None):
            self._np_random = _pcg(seed)
            return [seed]

        def sample(self):
            s = self.np_random.uniform(low=self.low, high=self.high, size=self.shape)
            return s.astype(self.dtype)

    spaces.Box = Box
    gym.Env = Env
    gym.spaces = spaces
    sys.modules["gymnasium"] = gym
    sys.modules["gymnasium.spaces"] = spaces


def stub_package(name):
    """Register a namespace for a reference package without running its
    __init__ (which would pull in matplotlib plotting modules)."""
    mod = types.ModuleType(name)
    mod.__path__ = [os.path.join(REF, name)]
    sys.modules[name] = mod


install_gym_standin()
sys.path.insert(0, REF)
stub_package("training")
stub_package("evaluation")

from envs import DexterousManipulationEnv  # noqa: E402
from experiments.config import CurriculumConfig  # noqa: E402
from experiments.curriculum_scheduler import CurriculumScheduler, StepBasedScheduler  # noqa: E402
from policies.simple_learner import SimpleLearner  # noqa: E402
from policies.random_policy import RandomPolicy  # noqa: E402
from training.episode_utils import run_episode  # noqa: E402
from evaluation.heldout_objects import HeldOutObjectSet, generate_training_objects  # noqa: E402
from evaluation.robustness_tests import CombinedNoiseWrapper  # noqa: E402

PRESETS = {
    "easy": CurriculumConfig.easy,
    "medium": CurriculumConfig.medium,
    "hard": CurriculumConfig.hard,
    "default": CurriculumConfig,
}


def make_cfg(name):
    if name == "variable":
        return CurriculumConfig.from_json(os.path.join(REF, "experiments", "config_variable.json"))
    if name == "interp":
        # scheduler interpolation -> numpy float64 size/mass/friction (NEP 50 quirk)
        s = CurriculumScheduler(CurriculumConfig.easy(), CurriculumConfig.hard())
        return s._interpolate_config(0.4)
    return PRESETS[name]()


def cfg_record(cfg):
    d = cfg.to_dict()
    out = {}
    for k, v in d.items():
        if isinstance(v, (tuple, list)):
            out[k] = [float(x) for x in v]
        elif v is None:
            out[k] = None
        else:
            out[k] = float(v)
    out["_float64_scalars"] = [k for k in ("object_size", "object_mass", "friction_coefficient")
                               if isinstance(getattr(cfg, k), np.floating)]
    return out


def replay_reset_draws(rng, cfg, first):
    """The draws reset() consumes, in order (manipulation_env.py:143-161)."""
    jp = rng.uniform(low=-0.1, high=0.1, size=(15,))
    size = mass = fric = np.nan
    if cfg.object_size_range is not None:
        size = float(rng.uniform(cfg.object_size_range[0], cfg.object_size_range[1]))
    if cfg.object_mass_range is not None:
        mass = float(rng.uniform(cfg.object_mass_range[0], cfg.object_mass_range[1]))
    if cfg.friction_range is not None:
        fric = float(rng.uniform(cfg.friction_range[0], cfg.friction_range[1]))
    spawn = np.full(3, np.nan)
    if first:
        spawn = np.array([float(rng.uniform(*cfg.spawn_x_range)),
                          float(rng.uniform(*cfg.spawn_y_range)),
                          float(rng.uniform(*cfg.spawn_z_range))])
    return np.concatenate([jp, [size, mass, fric], spawn])


# --------------------------------------------------------------------------
# 1. env reset/step traces (A2-A7)
# --------------------------------------------------------------------------
ENV_CASES = [
    dict(cfg="easy", reward="dense", seed=42, E=3, T=120, mode="uniform"),
    dict(cfg="medium", reward="dense", seed=7, E=3, T=120, mode="uniform"),
    dict(cfg="hard", reward="dense", seed=123, E=3, T=120, mode="drift"),
    dict(cfg="variable", reward="dense", seed=5, E=4, T=120, mode="uniform"),
    dict(cfg="variable", reward="sparse", seed=11, E=3, T=80, mode="uniform"),
    dict(cfg="hard", reward="sparse", seed=0, E=2, T=60, mode="drift"),
    dict(cfg="default", reward="dense", seed=3, E=2, T=40, mode="uniform", max_episode_steps=30),
    dict(cfg="easy", reward="dense", seed=9, E=3, T=60, mode="uniform", object_position=[0.01, -0.02, 0.1]),
    dict(cfg="interp", reward="dense", seed=21, E=2, T=100, mode="drift"),
    dict(cfg="variable", reward="dense", seed=2024, E=2, T=210, mode="drift"),
]
for s in range(8):
    ENV_CASES.append(dict(cfg=["easy", "medium", "hard", "variable"][s % 4], reward="dense",
                          seed=100 + s, E=2, T=100, mode="uniform" if s < 4 else "drift"))


def action_tape(mode, seed, E, T):
    r = np.random.default_rng(10_000 + seed)
    if mode == "uniform":
        return r.uniform(-1.3, 1.3, size=(E, T, 15)).astype(np.float32)
    base = r.uniform(-1.2, 1.2, size=(E, 1, 15))
    return (base + r.normal(0, 0.2, size=(E, T, 15))).astype(np.float32)


def gen_env_traces():
    arrays = {}
    meta = []
    for ci, c in enumerate(ENV_CASES):
        cfg = make_cfg(c["cfg"])
        mes = c.get("max_episode_steps", 200)
        env = DexterousManipulationEnv(
            reward_type=c["reward"], curriculum_config=cfg, max_episode_steps=mes,
            object_position=None if c.get("object_position") is None
            else np.array(c["object_position"]))
        E, T = c["E"], c["T"]
        acts = action_tape(c["mode"], c["seed"], E, T)
        twin = _pcg(c["seed"])
        first = c.get("object_position") is None
        R = dict(reset_obs=np.zeros((E, 45), np.float32), reset_op=np.zeros((E, 3)),
                 reset_params=np.zeros((E, 3)), reset_ncon=np.zeros(E, np.int32),
                 reset_has_comps=np.zeros(E, np.uint8), draws=np.zeros((E, 21)),
                 actions=acts, obs=np.zeros((E, T, 45), np.float32), reward=np.zeros((E, T)),
                 comps=np.zeros((E, T, 4)), term=np.zeros((E, T), np.uint8),
                 trunc=np.zeros((E, T), np.uint8), ncon=np.zeros((E, T), np.int32),
                 op=np.zeros((E, T, 3)), step_count=np.zeros((E, T), np.int32),
                 length=np.zeros(E, np.int32))
        for e in range(E):
            R["draws"][e] = replay_reset_draws(twin, cfg, first)
            obs, info = env.reset(seed=c["seed"] if e == 0 else None)
            first = False
            assert np.array_equal(env.joint_positions, R["draws"][e][:15].astype(np.float32))
            R["reset_obs"][e] = obs
            R["reset_op"][e] = np.asarray(info["object_position"], np.float64)
            cur = info["curriculum"]
            R["reset_params"][e] = [cur["object_size"], cur["object_mass"], cur["friction_coefficient"]]
            R["reset_ncon"][e] = info["num_contacts"]
            R["reset_has_comps"][e] = "reward_components" in info
            n = 0
            for t in range(T):
                obs, rew, term, trunc, info = env.step(acts[e, t])
                rc = info["reward_components"]
                R["obs"][e, t] = obs
                R["reward"][e, t] = rew
                R["comps"][e, t] = [rc["distance"], rc["contact"], rc["closure"], rc["stability"]]
                R["term"][e, t] = bool(term)
                R["trunc"][e, t] = bool(trunc)
                R["ncon"][e, t] = info["num_contacts"]
                R["op"][e, t] = np.asarray(info["object_position"], np.float64)
                R["step_count"][e, t] = info["step_count"]
                n = t + 1
                if term or trunc:
                    break
            R["length"][e] = n
        for k, v in R.items():
            arrays[f"c{ci}_{k}"] = v
        meta.append(dict(c, index=ci, max_episode_steps=mes, curriculum=cfg_record(cfg)))
    np.savez_compressed(os.path.join(OUT, "env_traces.npz"), **arrays)
    return meta


# --------------------------------------------------------------------------
# 2. run_episode + SimpleLearner (A8/A9); RandomPolicy plumbing (C1)
# --------------------------------------------------------------------------
LEARNER_CASES = [
    dict(cfg="easy", reward="dense", learner_seed=42, env_seed=1000, episodes=5, max_steps=200, lr=0.01),
    dict(cfg="hard", reward="dense", learner_seed=123, env_seed=2000, episodes=3, max_steps=200, lr=0.01),
    dict(cfg="variable", reward="dense", learner_seed=7, env_seed=3000, episodes=4, max_steps=200, lr=0.05),
    dict(cfg="medium", reward="sparse", learner_seed=5, env_seed=4000, episodes=3, max_steps=200, lr=0.01),
    dict(cfg="default", reward="dense", learner_seed=456, env_seed=5000, episodes=4, max_steps=100, lr=0.01),
    dict(cfg="hard", reward="dense", learner_seed=789, env_seed=6000, episodes=2, max_steps=200, lr=0.01,
         max_episode_steps=50),
]


def gen_learner_traces():
    arrays = {}
    meta = []
    for ci, c in enumerate(LEARNER_CASES):
        cfg = make_cfg(c["cfg"])
        env = DexterousManipulationEnv(reward_type=c["reward"], curriculum_config=cfg,
                                       max_episode_steps=c.get("max_episode_steps", 200))
        env.np_random = _pcg(c["env_seed"])  # entropy-seeded in the drivers; fixed here
        np.random.seed(c["learner_seed"])  # as evaluation/component_ablation.py:99
        pol = SimpleLearner(env.action_space, learning_rate=c["lr"])
        rec = dict(action=[], reward=[], mean=[], best=[], term=[], trunc=[])
        orig_step, orig_select, orig_update = env.step, pol.select_action, pol.update

        def step(a, _s=orig_step):
            o, r, te, tr, i = _s(a)
            rec["reward"].append(r)
            rec["term"].append(te)
            rec["trunc"].append(tr)
            return o, r, te, tr, i

        def select(o, _s=orig_select):
            a = _s(o)
            rec["action"].append(a.copy())
            return a

        def update(r, _u=orig_update):
            _u(r)
            rec["mean"].append(pol.mean_action.copy())
            rec["best"].append(pol.best_reward)

        env.step, pol.select_action, pol.update = step, select, update
        ep = []
        for _ in range(c["episodes"]):
            ep.append(run_episode(env, pol, max_steps=c["max_steps"]))
        arrays[f"l{ci}_action"] = np.array(rec["action"], np.float32)
        arrays[f"l{ci}_reward"] = np.array(rec["reward"])
        arrays[f"l{ci}_mean"] = np.array(rec["mean"], np.float32)
        arrays[f"l{ci}_best"] = np.array(rec["best"])
        arrays[f"l{ci}_term"] = np.array(rec["term"], np.uint8)
        arrays[f"l{ci}_trunc"] = np.array(rec["trunc"], np.uint8)
        arrays[f"l{ci}_ep_success"] = np.array([e[0] for e in ep], np.uint8)
        arrays[f"l{ci}_ep_steps"] = np.array([e[1] for e in ep], np.int32)
        arrays[f"l{ci}_ep_return"] = np.array([e[2] for e in ep])
        arrays[f"l{ci}_final_mean"] = pol.mean_action.copy()
        meta.append(dict(c, index=ci, curriculum=cfg_record(cfg)))

    # C1 plumbing: config_quick_test-like RandomPolicy episodes, default curriculum
    env = DexterousManipulationEnv(reward_type="dense", max_episode_steps=100)
    env.np_random = _pcg(77)
    pol = RandomPolicy(env.action_space, seed=42)
    env.action_space.seed(4242)  # the reference never seeds Box.sample (entropy); fixed here
    rets = [run_episode(env, pol) for _ in range(3)]
    arrays["rp_ep_success"] = np.array([r[0] for r in rets], np.uint8)
    arrays["rp_ep_steps"] = np.array([r[1] for r in rets], np.int32)
    arrays["rp_ep_return"] = np.array([r[2] for r in rets])
    np.savez_compressed(os.path.join(OUT, "learner_traces.npz"), **arrays)
    return meta, dict(env_seed=77, box_seed=4242, max_episode_steps=100, episodes=3)


# --------------------------------------------------------------------------
# 3. CombinedNoiseWrapper (A10) as RobustnessTester drives it
# --------------------------------------------------------------------------
NOISE_CASES = [
    dict(cfg="variable", obs_std=0.05, dyn_std=0.05, seed=42, episodes=3, T=100),
    dict(cfg="hard", obs_std=0.05, dyn_std=0.0, seed=7, episodes=2, T=80),
    dict(cfg="easy", obs_std=0.0, dyn_std=0.1, seed=3, episodes=2, T=80),
]


def gen_noise_traces():
    arrays = {}
    for ci, c in enumerate(NOISE_CASES):
        cfg = make_cfg(c["cfg"])
        base = DexterousManipulationEnv(curriculum_config=cfg, reward_type="dense", max_episode_steps=200)
        env = CombinedNoiseWrapper(base, c["obs_std"], c["dyn_std"], seed=c["seed"])
        E, T = c["episodes"], c["T"]
        acts = action_tape("uniform", 500 + ci, E, T)
        obs_r = np.zeros((E, T, 45), np.float32)
        rew = np.zeros((E, T))
        reset_obs = np.zeros((E, 45), np.float32)
        length = np.zeros(E, np.int32)
        for e in range(E):
            o, _ = env.reset(seed=c["seed"] + e)  # robustness_tests.py:281-282
            reset_obs[e] = o
            for t in range(T):
                o, r, te, tr, _ = env.step(acts[e, t])
                obs_r[e, t] = o
                rew[e, t] = r
                length[e] = t + 1
                if te or tr:
                    break
        arrays.update({f"n{ci}_actions": acts, f"n{ci}_obs": obs_r, f"n{ci}_reward": rew,
                       f"n{ci}_reset_obs": reset_obs, f"n{ci}_length": length})
    np.savez_compressed(os.path.join(OUT, "noise_traces.npz"), **arrays)
    return NOISE_CASES


# --------------------------------------------------------------------------
# 4. held-out object tables (A15) and curriculum scheduler traces (A14)
# --------------------------------------------------------------------------
def gen_host_tables():
    out = {"heldout": [], "training_objects": [], "scheduler": [], "configs": {}}
    for cfg_name, n, seed in [("hard", 10, 42), ("variable", 20, 123), ("easy", 5, 42), ("medium", 10, 7)]:
        h = HeldOutObjectSet(make_cfg(cfg_name), num_heldout_objects=n, seed=seed)
        out["heldout"].append(dict(
            cfg=cfg_name, n=n, seed=seed, eval_size_range=list(h.eval_size_range),
            eval_mass_range=list(h.eval_mass_range), eval_friction_range=list(h.eval_friction_range),
            objects=[[o.size, o.mass, o.friction] for o in h.heldout_objects],
            eval_configs=[cfg_record(h.get_eval_config(i)) for i in range(n + 2)],
            statistics=h.get_statistics()))
    objs = generate_training_objects(make_cfg("variable"), num_samples=50, seed=42)
    out["training_objects"] = [[o.size, o.mass, o.friction] for o in objs]

    rng = np.random.default_rng(99)
    sched_cases = [
        dict(kind="success", thr=0.3, window=15, min_eps=20, steps=5, p=[0.0] * 40 + [0.5] * 80 + [0.9] * 80),
        dict(kind="success", thr=0.7, window=20, min_eps=50, steps=3, p=[0.8] * 200),
        dict(kind="success", thr=0.3, window=10, min_eps=10, steps=3, p=[0.2] * 30 + [0.6] * 60),
    ]
    for sc in sched_cases:
        s = CurriculumScheduler(CurriculumConfig.easy(), CurriculumConfig.hard(),
                                success_rate_threshold=sc["thr"], window_size=sc["window"],
                                min_episodes_before_progression=sc["min_eps"], progression_steps=sc["steps"])
        succ = [bool(rng.random() < p) for p in sc["p"]]
        steps = [int(rng.integers(1, 201)) for _ in sc["p"]]
        progressed, levels, cfgs = [], [], []
        for a, b in zip(succ, steps):
            progressed.append(bool(s.update(a, b)))
            levels.append(float(s.get_difficulty_level()))
            cfgs.append(cfg_record(s.get_current_config()))
        stats = s.get_statistics()
        out["scheduler"].append(dict(sc, successes=succ, steps_seq=steps, progressed=progressed,
                                     levels=levels, configs=cfgs, statistics=stats))
    # step-based scheduler
    s = StepBasedScheduler(CurriculumConfig.easy(), CurriculumConfig.hard(), step_milestones=[500, 100, 1500])
    steps = [int(rng.integers(1, 201)) for _ in range(30)]
    prog = [bool(s.update(False, b)) for b in steps]
    out["step_scheduler"] = dict(milestones=[500, 100, 1500], steps_seq=steps, progressed=prog,
                                 statistics=s.get_statistics(), final=cfg_record(s.get_current_config()))
    for name in ["easy", "medium", "hard", "variable", "default", "interp"]:
        out["configs"][name] = cfg_record(make_cfg(name))
    for fname in ["config_easy.json", "config_medium.json", "config_hard.json", "config_variable.json",
                  "config_default.json", "config_quick_test.json"]:
        with open(os.path.join(REF, "experiments", fname)) as f:
            out["configs"]["json:" + fname] = json.load(f)
    return out


def main():
    meta = {"generator": "tests/golden/gen_golden.py", "numpy": np.__version__}
    meta["env_cases"] = gen_env_traces()
    meta["learner_cases"], meta["random_policy"] = gen_learner_traces()
    meta["noise_cases"] = gen_noise_traces()
    meta["host"] = gen_host_tables()
    with open(os.path.join(OUT, "golden_meta.json"), "w") as f:
        json.dump(meta, f, indent=1, default=float)
    print("wrote fixtures to", OUT)


if __name__ == "__main__":
    main()
